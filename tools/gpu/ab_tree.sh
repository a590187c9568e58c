#!/bin/bash
# Same-session A/B of two whole source trees (Python + their own built extension): the current
# tree against an older checkout staged (built) under ab_tree/ — for changes that touch both the
# kernels and the Python call sites, where swapping only the .so (ab_build.sh) cannot work.
#   CFGS="resnet50:256 vgg11:256 vgg11:32" bash tools/gpu/ab_tree.sh
cd "$GRAFT_REPO_ROOT" || exit 2
OUT=$GRAFT_REPO_ROOT/gpurun_out/ab_tree
mkdir -p $OUT
CFGS=${CFGS:-"resnet50:256 vgg11:256 vgg11:32"}
for P in 1 2; do
  for CFG in $CFGS; do
    M=${CFG%%:*}; B=${CFG##*:}; S=60; [ $M = resnet50 ] && S=20
    for T in old cur; do
      D=$GRAFT_REPO_ROOT; [ $T = old ] && D=$GRAFT_REPO_ROOT/ab_tree
      L=$OUT/${M}_b${B}_${T}_p$P.log
      (cd $D && timeout -k 10 240 python bench.py --model $M --global-batch $B --steps $S --warmup 10 --ref-window 0 > $L 2>&1) || { tail -5 $L; exit 1; }
      echo "$M B=$B $T p$P $(python -c "import json; d=json.loads(open('$L').read().strip().splitlines()[-1]); print(d['ms_per_step'])")"
    done
  done
done
