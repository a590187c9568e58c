#!/bin/bash
# round 4: BN-backward sums fusion threshold (DDP_AMD_BN_BWD_FUSE_MAX_HW) across per-GPU batches
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r4z; mkdir -p $O
for B in 256 128 32; do
  if [ $B = 32 ]; then L="16 256 16 256"; else L="16 64 16 64"; fi
  for hw in $L; do
  timeout -k 10 200 env DDP_AMD_BN_BWD_FUSE_MAX_HW=$hw python bench.py --global-batch $B --steps 60 --warmup 10 --ref-window 0 > $O/b${B}_hw${hw}.log 2>&1 || { tail -5 $O/b${B}_hw${hw}.log; exit 1; }
  echo "b$B hw$hw $(tail -1 $O/b${B}_hw${hw}.log | grep -oE '"ms_per_step": [0-9.]+')"
done; done
