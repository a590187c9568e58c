#!/bin/bash
# A/B of an environment knob on the 1-GPU bench: bash tools/gpu_ab.sh VAR "v1 v2 ..." [model]
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
var=$1; vals=$2; model=${3:-vgg11}
for v in $vals; do
  env "$var=$v" timeout -k 10 300 python bench.py --model "$model" --steps 40 --warmup 10 > "gpurun_out/ab_${var}_${v}_${model}.log" 2>&1
  rc=$?
  echo "$var=$v rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_${var}_${v}_${model}.log)"
  [ $rc -ne 0 ] && tail -5 "gpurun_out/ab_${var}_${v}_${model}.log" && exit $rc
done
exit 0
