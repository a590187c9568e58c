#!/bin/bash
# ResNet-50 bench loss at lr 0 / 0.001, graph replay vs eager steps, repeated processes.
cd "$GRAFT_REPO_ROOT" || exit 2
OUT=$GRAFT_REPO_ROOT/gpurun_out/gspike
mkdir -p $OUT
for R in $(seq 1 ${RUNS:-3}); do
  for V in "lr0:--lr 0" "lr0_eager:--lr 0 --no-graph" "lr1e-3_eager:--lr 0.001 --no-graph"; do
    N=${V%%:*}; A=${V#*:}
    L=$OUT/${N}_r$R.log
    timeout -k 10 240 python bench.py --model resnet50 --steps 12 --warmup 4 --ref-window 0 $A > $L 2>&1 || { tail -5 $L; exit 1; }
    echo "$N r$R $(python -c "import json; d=json.loads(open('$L').read().strip().splitlines()[-1]); print(d['train_loss_mean'], d['warmup_loss_sum'])")"
  done
done
