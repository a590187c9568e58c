#!/bin/bash
# round 5: grid caps re-checked on the current kernels (no rebuild): FWD-GEMM statistics grid
# (DDP_AMD_FWD_STAT_GRID) and BN-backward reduce grid (DDP_AMD_BN_REDUCE_GRID), ResNet-50 b256
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r5ao; mkdir -p $O
for i in 1 2; do
  for cfg in "F=2048 R=2048" "F=1024 R=2048" "F=4096 R=2048" "F=2048 R=4096" "F=2048 R=1024"; do
    eval $cfg
    DDP_AMD_FWD_STAT_GRID=$F DDP_AMD_BN_REDUCE_GRID=$R timeout -k 10 300 python bench.py --model resnet50 --steps 8 --warmup 4 --ref-window 0 > $O/r_${F}_${R}_$i.log 2>&1 || { tail -5 $O/r_${F}_${R}_$i.log; exit 1; }
    tail -1 $O/r_${F}_${R}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('fwd_grid=$F reduce_grid=$R', d['ms_per_step'], d['value'])"
  done
done
