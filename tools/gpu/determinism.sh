#!/bin/bash
# Run-to-run spread of the bench loss per environment variant (same seeds, same data: the only
# differences between runs are float-atomic arrival orders). A variant whose spread is far above
# the others points at a race.
#   VARIANTS="a:X=0 b:X=1" CFGS="resnet50:256 vgg11:256" RUNS=3 bash tools/gpu/determinism.sh
cd "$GRAFT_REPO_ROOT" || exit 2
OUT=gpurun_out/determinism
mkdir -p $OUT
RUNS=${RUNS:-3}
for CFG in ${CFGS:-resnet50:256}; do
  M=${CFG%%:*}; B=${CFG##*:}; S=30; [ $M = resnet50 ] && S=15
  for V in $VARIANTS; do
    NAME=${V%%:*}; ENVS=${V#*:}
    for R in $(seq 1 $RUNS); do
      L=$OUT/${M}_b${B}_${NAME}_r$R.log
      env ${ENVS//,/ } timeout -k 10 240 python bench.py --model $M --global-batch $B --steps $S --warmup 5 --ref-window 0 --lr 0.01 > $L 2>&1 || { tail -5 $L; exit 1; }
      echo "$M B=$B $NAME r$R $(python -c "import json; d=json.loads(open('$L').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['train_loss_mean'], d['warmup_loss_sum'])")"
    done
  done
done
