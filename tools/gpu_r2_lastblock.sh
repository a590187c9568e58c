#!/bin/bash
# BN-backward in-launch finalize (reduce kernel's last block) vs separate finalize, per batch
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/lb
for P in 1 2; do
for B in 32 64 128 256; do
  for V in 0 1; do
    L=gpurun_out/lb/b${B}_$V_p$P.log
    DDP_AMD_BN_LAST_BLOCK=$V timeout -k 10 120 python bench.py --global-batch $B --steps 60 --warmup 10 --ref-window 0 > $L 2>&1 || { tail -5 $L; exit 1; }
    echo "B=$B last_block=$V p$P $(python -c "import json; d=json.loads(open('$L').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['train_loss_mean'])")"
  done
done
done
