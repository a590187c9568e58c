#!/bin/bash
# round 5: BN finalize folded into the apply (bn_act.hip: backward FOLD, DDP_AMD_BN_FOLD_BWD_MB;
# forward capped-grid FOLD, DDP_AMD_BN_FOLD_FWD_GRID)
# — BN kernel tests, model tests, VGG-11 b256 / b32 and ResNet-50 A/B (0 = separate finalize)
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r5v; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py -k "bn_act or linear_head or splitk or finish or deferred" tests/test_gpu_model.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAIL|Error" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for b in 256 32; do
  for i in 1 2 3; do
    for m in 0 32; do
      DDP_AMD_BN_FOLD_BWD_MB=$m timeout -k 10 200 python bench.py --global-batch $b --steps 60 --warmup 10 > $O/vgg_b${b}_f${m}_$i.log 2>&1 || { tail -5 $O/vgg_b${b}_f${m}_$i.log; exit 1; }
      tail -1 $O/vgg_b${b}_f${m}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('b$b fold=$m', d['ms_per_step'], d['value'])"
    done
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_resnet.py -x -q --timeout 300 --timeout-method thread > $O/tests_r.log 2>&1 || { tail -30 $O/tests_r.log; exit 1; }
tail -1 $O/tests_r.log
for i in 1 2; do
  for m in 0 1; do
    if [ $m = 0 ]; then F="DDP_AMD_BN_FOLD_BWD_MB=0 DDP_AMD_BN_FOLD_FWD_GRID=0"; else F="DDP_AMD_BN_FOLD_BWD_MB=32"; fi
    env $F timeout -k 10 300 python bench.py --model resnet50 --steps 8 --warmup 4 --ref-window 0 > $O/resnet_f${m}_$i.log 2>&1 || { tail -5 $O/resnet_f${m}_$i.log; exit 1; }
    tail -1 $O/resnet_f${m}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('resnet fold=$m', d['ms_per_step'], d['value'])"
  done
done
