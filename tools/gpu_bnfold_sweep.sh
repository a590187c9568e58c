#!/bin/bash
# BN-backward finalize fold threshold sweep (DDP_AMD_BN_FOLD_BWD_KB), VGG-11 b256, 1 GPU.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
for kb in 0 1100 4200 8400 0; do
  DDP_AMD_BN_FOLD_BWD_KB=$kb timeout -k 10 200 python bench.py --steps 200 --warmup 20 > gpurun_out/fold.log 2>&1 || { echo "kb=$kb FAILED"; tail -5 gpurun_out/fold.log; exit 1; }
  echo "fold_kb=$kb $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/fold.log)"
done
