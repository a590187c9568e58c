#!/bin/bash
# World-1 "overlapped optimizer": the pipelined step without a collective (per-segment SGD on the
# high-priority stream while earlier layers back-propagate) vs the single-graph step
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/oo
for P in 1 2; do
for B in 256 32; do
  for C in 0 5 6 4,6 3,6 2,5; do
    L=gpurun_out/oo/b${B}_c${C}_p$P.log
    timeout -k 10 120 python bench.py --global-batch $B --steps 60 --warmup 10 --ref-window 0 --segmented $C > $L 2>&1 || { tail -5 $L; exit 1; }
    echo "B=$B cuts=$C p$P $(python -c "import json; d=json.loads(open('$L').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['train_loss_mean'])")"
  done
done
done
