#!/bin/bash
# round 5: BN-backward finalize folded into small-grid applies only (capped-grid folds off):
# ResNet-50 b256 and VGG-11 b32 / b256 A/B (DDP_AMD_BN_FOLD_BWD_MB=0 vs default 32)
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r5w; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -k "bn_act" -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for m in 0 32; do
    DDP_AMD_BN_FOLD_BWD_MB=$m timeout -k 10 300 python bench.py --model resnet50 --steps 8 --warmup 4 --ref-window 0 > $O/resnet_f${m}_$i.log 2>&1 || { tail -5 $O/resnet_f${m}_$i.log; exit 1; }
    tail -1 $O/resnet_f${m}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('resnet fold=$m', d['ms_per_step'], d['value'])"
  done
done
for b in 32 256; do
  for i in 1 2 3; do
    for m in 0 32; do
      DDP_AMD_BN_FOLD_BWD_MB=$m timeout -k 10 200 python bench.py --global-batch $b --steps 60 --warmup 10 > $O/vgg_b${b}_f${m}_$i.log 2>&1 || { tail -5 $O/vgg_b${b}_f${m}_$i.log; exit 1; }
      tail -1 $O/vgg_b${b}_f${m}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('b$b fold=$m', d['ms_per_step'], d['value'])"
    done
  done
done
