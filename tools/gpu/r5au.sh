#!/bin/bash
# round 5: ResNet-50 tuning gaps — the stride-1 3x3 convs of layer2..4's non-first blocks were
# missing from the tuned layer list (their DGRAD ran the cost-model tile), and the backward pair
# (DGRAD + WGRAD in one launch, mode-3 entries) was never tuned for ResNet. Tune DGRAD, then the
# pairs, then A/B the step with the old and the new table in the same session.
cd "$GRAFT_REPO_ROOT" || exit 2
OUT=gpurun_out/tune5; mkdir -p $OUT
TABLE=distributed-data-parallel-ml-training_amd/ops/conv_tuning.json
cp $TABLE $OUT/old.json
timeout -k 10 600 python -u tools/conv_tune.py --sets resnet256 --modes dgrad --reps 20 \
    --merge $OUT/old.json --out $OUT/mid.json > $OUT/tune_dgrad.log 2>&1 || { tail -20 $OUT/tune_dgrad.log; cp $OUT/old.json $TABLE; exit 1; }
tail -2 $OUT/tune_dgrad.log
cp $OUT/mid.json $TABLE
timeout -k 10 600 python -u tools/conv_tune.py --pairs --pair-sets resnet50:256 --reps 20 \
    --merge $OUT/mid.json --out $OUT/new.json > $OUT/tune_pairs.log 2>&1 || { tail -20 $OUT/tune_pairs.log; cp $OUT/old.json $TABLE; exit 1; }
tail -2 $OUT/tune_pairs.log
for P in 1 2; do
  for T in old mid new; do
    cp $OUT/$T.json $TABLE
    L=$OUT/resnet_${T}_p$P.log
    timeout -k 10 240 python bench.py --model resnet50 --steps 20 --warmup 10 --ref-window 0 > $L 2>&1 || { tail -5 $L; cp $OUT/old.json $TABLE; exit 1; }
    echo "resnet50 table=$T p$P $(python -c "import json; d=json.loads(open('$L').read().strip().splitlines()[-1]); print(d['ms_per_step'])")"
  done
done
for T in old new; do
  cp $OUT/$T.json $TABLE
  for b in 256 32; do
    L=$OUT/vgg_b${b}_$T.log
    timeout -k 10 200 python bench.py --global-batch $b --steps 60 --warmup 10 > $L 2>&1 || { tail -5 $L; cp $OUT/old.json $TABLE; exit 1; }
    echo "vgg11 b$b table=$T $(python -c "import json; d=json.loads(open('$L').read().strip().splitlines()[-1]); print(d['ms_per_step'])")"
  done
done
cp $OUT/old.json $TABLE
