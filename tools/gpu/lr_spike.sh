#!/bin/bash
# Divergence rate of the ResNet-50 bench vs learning rate (current tree): chaotic dynamics fade
# with the lr, a race does not.
cd "$GRAFT_REPO_ROOT" || exit 2
OUT=$GRAFT_REPO_ROOT/gpurun_out/lrspike
mkdir -p $OUT
for R in $(seq 1 ${RUNS:-4}); do
  for LR in ${LRS:-0.001 0.01}; do
    L=$OUT/lr${LR}_r$R.log
    timeout -k 10 240 python bench.py --model resnet50 --steps 20 --warmup 5 --ref-window 0 --lr $LR > $L 2>&1 || { tail -5 $L; exit 1; }
    echo "lr $LR r$R $(python -c "import json; d=json.loads(open('$L').read().strip().splitlines()[-1]); print(d['train_loss_mean'], d['warmup_loss_sum'])")"
  done
done
