#!/bin/bash
# round 5: FWD GEMM statistics accumulated across a capped grid's work items
# (conv_igemm.hip run_s / flush_stats, DDP_AMD_FWD_STAT_GRID) — conv kernel tests, ResNet
# tests, deterministic test, ResNet-50 b256 and VGG-11 b256 A/B (0 = one block per item)
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r5u; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_deterministic.py -x -q --timeout 300 --timeout-method thread > $O/tests_k.log 2>&1 || { grep -E "FAIL|Error" $O/tests_k.log | head; tail -30 $O/tests_k.log; exit 1; }
tail -1 $O/tests_k.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_resnet.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAIL|Error" $O/tests.log | head -20; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for m in 0 2048; do
    DDP_AMD_FWD_STAT_GRID=$m timeout -k 10 300 python bench.py --model resnet50 --steps 8 --warmup 4 --ref-window 0 > $O/resnet_g${m}_$i.log 2>&1 || { tail -5 $O/resnet_g${m}_$i.log; exit 1; }
    tail -1 $O/resnet_g${m}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('resnet grid=$m', d['ms_per_step'], d['value'], d['train_loss_mean'])"
  done
done
for i in 1 2; do
  for m in 0 2048; do
    DDP_AMD_FWD_STAT_GRID=$m timeout -k 10 200 python bench.py --steps 60 --warmup 10 > $O/vgg_g${m}_$i.log 2>&1 || { tail -5 $O/vgg_g${m}_$i.log; exit 1; }
    tail -1 $O/vgg_g${m}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('vgg grid=$m', d['ms_per_step'], d['value'])"
  done
done
