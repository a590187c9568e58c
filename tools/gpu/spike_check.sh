#!/bin/bash
# ResNet-50 bench loss over repeated runs, old tree (ab_tree/) vs current tree: does either
# diverge (train_loss_mean far above ln(1000) or NaN) more often?
cd "$GRAFT_REPO_ROOT" || exit 2
OUT=$GRAFT_REPO_ROOT/gpurun_out/spike
mkdir -p $OUT
for R in $(seq 1 ${RUNS:-4}); do
  for T in old cur; do
    D=$GRAFT_REPO_ROOT; [ $T = old ] && D=$GRAFT_REPO_ROOT/ab_tree
    L=$OUT/${T}_r$R.log
    (cd $D && timeout -k 10 240 python bench.py --model resnet50 --steps 20 --warmup 5 --ref-window 0 > $L 2>&1) || { tail -5 $L; exit 1; }
    echo "$T r$R $(python -c "import json; d=json.loads(open('$L').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['train_loss_mean'], d['warmup_loss_sum'])")"
  done
done
