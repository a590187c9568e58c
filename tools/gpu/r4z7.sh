#!/bin/bash
# round 4: re-tune the backward-pair table for the 4- / 8-GPU shares (their 16x16 / 8x8 dgrads now
# carry the BN-backward sums), then A/B old vs new table in the same session
cd "$GRAFT_REPO_ROOT" || exit 2
OUT=gpurun_out/r4z7; mkdir -p $OUT
TABLE=distributed-data-parallel-ml-training_amd/ops/conv_tuning.json
cp $TABLE $OUT/old.json
timeout -k 10 600 python -u tools/conv_tune.py --pairs --pair-sets vgg11:32,64 --reps 40 \
    --merge $OUT/old.json --out $OUT/new.json > $OUT/tune.log 2>&1 || { tail -20 $OUT/tune.log; exit 1; }
cat $OUT/tune.log | grep -v amdgpu.ids
for P in 1 2; do for T in old new; do
  cp $OUT/$T.json $TABLE
  for B in 64 32; do
    L=$OUT/b${B}_${T}_p$P.log
    timeout -k 10 200 python bench.py --global-batch $B --steps 60 --warmup 10 --ref-window 0 > $L 2>&1 || { tail -5 $L; cp $OUT/old.json $TABLE; exit 1; }
    echo "b$B $T p$P $(tail -1 $L | grep -oE '"ms_per_step": [0-9.]+')"
  done
done; done
cp $OUT/old.json $TABLE
