#!/bin/bash
# Same-session A/B of native-extension builds: in-tree ("cur") vs ab_so/_native_<name>.so.
#   VARIANTS="old cur" PROF=1 bash tools/gpu/ab_build.sh
# Benches interleaved over two passes; PROF=1 adds a rocprofv3 --stats run of VGG-11 b256 and
# b32 per variant (kernel tables under gpurun_out/ab_var/prof_<variant>_b<batch>/).
cd "$GRAFT_REPO_ROOT" || exit 2
OUT=gpurun_out/ab_var
mkdir -p $OUT
VARIANTS=${VARIANTS:-"old cur"}
CFGS=${CFGS:-"vgg11:256 vgg11:32 resnet50:256"}
sel() { if [ "$1" = cur ]; then echo ""; else echo "ab_so/_native_$1.so"; fi; }
for P in 1 2; do
  for CFG in $CFGS; do
    M=${CFG%%:*}; B=${CFG##*:}; S=60; [ $M = resnet50 ] && S=20
    for V in $VARIANTS; do
      L=$OUT/${M}_b${B}_${V}_p$P.log
      DDP_AMD_NATIVE_PATH=$(sel $V) timeout -k 10 240 python bench.py --model $M --global-batch $B --steps $S --warmup 10 --ref-window 0 > $L 2>&1 || { tail -5 $L; exit 1; }
      echo "$M B=$B $V p$P $(python -c "import json; d=json.loads(open('$L').read().strip().splitlines()[-1]); print(d['ms_per_step'])")"
    done
  done
done
if [ -n "$PROF" ]; then
  for V in $VARIANTS; do
    for B in 256 32; do
      D=$GRAFT_REPO_ROOT/$OUT/prof_${V}_b$B
      (cd /tmp && export TMPDIR=/tmp && DDP_AMD_NATIVE_PATH=$(sel $V | sed "s|^ab_so|$GRAFT_REPO_ROOT/ab_so|") timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o p -- python3 $GRAFT_REPO_ROOT/bench.py --global-batch $B --steps 20 --warmup 5 --ref-window 0 > $D.log 2>&1) || { tail -5 $D.log; exit 1; }
    done
  done
  echo profiled
fi
