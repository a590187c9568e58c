#!/bin/bash
# round 5: ResNet table A/B — old, the r5au re-tune (new), and the re-tune with the three
# accumulate-mode DGRAD entries of r5o kept (new2; the plain-mode sweep had replaced them)
cd "$GRAFT_REPO_ROOT" || exit 2
OUT=_scratch; mkdir -p gpurun_out/tune5
TABLE=distributed-data-parallel-ml-training_amd/ops/conv_tuning.json
cp $TABLE $OUT/cur.json
for P in 1 2; do
  for T in old new new2; do
    cp $OUT/$T.json $TABLE
    L=gpurun_out/tune5/ab_${T}_p$P.log
    timeout -k 10 240 python bench.py --model resnet50 --steps 20 --warmup 10 --ref-window 0 > $L 2>&1 || { tail -5 $L; cp $OUT/cur.json $TABLE; exit 1; }
    echo "resnet50 table=$T p$P $(python -c "import json; d=json.loads(open('$L').read().strip().splitlines()[-1]); print(d['ms_per_step'])")"
  done
done
cp $OUT/cur.json $TABLE
