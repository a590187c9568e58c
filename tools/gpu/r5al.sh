#!/bin/bash
# round 5: projection-shortcut BatchNorm folded into the residual block's BN passes (bn_act.hip
# RBN, ops/layers.py RES_BN_FUSE) — kernel numerics, ResNet tests, ResNet-50 b256 A/B
# (DDP_AMD_RES_BN_FUSE=0 vs 1, interleaved), kernel profile of the new default
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r5al; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -k "bn_act" -x -q --timeout 300 --timeout-method thread > $O/tests_k.log 2>&1 || { tail -30 $O/tests_k.log; exit 1; }
tail -1 $O/tests_k.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_resnet.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAIL|Error" $O/tests.log | head -20; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for m in 0 1; do
    DDP_AMD_RES_BN_FUSE=$m timeout -k 10 300 python bench.py --model resnet50 --steps 8 --warmup 4 --ref-window 0 > $O/resnet_f${m}_$i.log 2>&1 || { tail -5 $O/resnet_f${m}_$i.log; exit 1; }
    tail -1 $O/resnet_f${m}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('fuse=$m', d['ms_per_step'], d['value'], d['train_loss_mean'])"
  done
done
TAG=r5al MODEL=resnet50 BATCHES=256 bash tools/gpu/profile.sh
