#!/bin/bash
# Re-tune the conv tile / split-K table for a model set with the current kernels, then bench the
# old table against the new one in the same session (the new table is left in gpurun_out/tune/).
#   SETS=resnet256 CFGS="resnet50:256" bash tools/gpu/retune.sh
cd "$GRAFT_REPO_ROOT" || exit 2
OUT=gpurun_out/tune
mkdir -p $OUT
TABLE=distributed-data-parallel-ml-training_amd/ops/conv_tuning.json
cp $TABLE $OUT/old.json
timeout -k 10 ${TUNE_S:-900} python -u tools/conv_tune.py --sets ${SETS:-resnet256} --modes ${MODES:-fwd,dgrad,wgrad} --reps ${REPS:-20} \
    --merge $OUT/old.json --out $OUT/new.json > $OUT/tune.log 2>&1 || { tail -20 $OUT/tune.log; exit 1; }
tail -3 $OUT/tune.log
for P in 1 2; do
  for T in old new; do
    cp $OUT/$T.json $TABLE
    for CFG in ${CFGS:-resnet50:256}; do
      M=${CFG%%:*}; B=${CFG##*:}; S=60; [ $M = resnet50 ] && S=20
      L=$OUT/${M}_b${B}_${T}_p$P.log
      timeout -k 10 240 python bench.py --model $M --global-batch $B --steps $S --warmup 10 --ref-window 0 > $L 2>&1 || { tail -5 $L; cp $OUT/old.json $TABLE; exit 1; }
      echo "$M B=$B table=$T p$P $(python -c "import json; d=json.loads(open('$L').read().strip().splitlines()[-1]); print(d['ms_per_step'])")"
    done
  done
done
cp $OUT/old.json $TABLE
