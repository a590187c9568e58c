#!/bin/bash
# A/B of conv tuning tables: shipped ops/conv_tuning.json vs the round-2 re-tune (r2) vs a merge
# (shipped entries, replaced where the re-tune measured >=5% faster). Interleaved, two passes.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/tuneab
for P in 1 2; do
for CFG in "vgg11 32" "vgg11 256" "vgg11 128" "vgg11 64" "resnet50 256"; do
  set -- $CFG; M=$1; B=$2
  for T in base merged r2; do
    case $T in base) F="";; *) F="tools/tune_cand/$T.json";; esac
    L=gpurun_out/tuneab/${M}_b${B}_${T}_p$P.log
    S=60; [ $M = resnet50 ] && S=20
    DDP_AMD_CONV_TUNING_FILE=${F:-distributed-data-parallel-ml-training_amd/ops/conv_tuning.json} \
      timeout -k 10 240 python bench.py --model $M --global-batch $B --steps $S --warmup 10 --ref-window 0 > $L 2>&1 || { tail -5 $L; exit 1; }
    echo "$M B=$B $T p$P $(python -c "import json; d=json.loads(open('$L').read().strip().splitlines()[-1]); print(d['ms_per_step'])")"
  done
done
done
