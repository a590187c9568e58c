#!/bin/bash
# BatchNorm forward / backward fused into the split-K finishes: numerics (kernel + model tests), then a
# same-session A/B (both off / forward only / both) at VGG-11 b32/b64/b128/b256, two passes,
# and a rocprofv3 kernel table of the b32 step.
cd "$GRAFT_REPO_ROOT" || exit 2
OUT=gpurun_out/bnfwd
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
CFGS=${CFGS:-"vgg11:32 vgg11:64 vgg11:128 vgg11:256"}
for P in 1 2; do
  for CFG in $CFGS; do
    M=${CFG%%:*}; B=${CFG##*:}; S=60; [ $M = resnet50 ] && S=20
    for V in ${VARS:-off fwd on}; do
      L=$OUT/${M}_b${B}_${V}_p$P.log
      F=1; BA=1; [ $V = off ] && F=0 && BA=0; [ $V = fwd ] && BA=0
      DDP_AMD_BN_FWD_FUSE=$F DDP_AMD_BN_BWD_APPLY_FUSE=$BA timeout -k 10 240 python bench.py --model $M --global-batch $B --steps $S --warmup 10 --ref-window 0 > $L 2>&1 || { tail -5 $L; exit 1; }
      echo "$M B=$B $V p$P $(python -c "import json; d=json.loads(open('$L').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['train_loss_mean'])")"
    done
  done
done
if [ -n "$PROF" ]; then
  D=$GRAFT_REPO_ROOT/$OUT/prof_b32
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o p -- python3 $GRAFT_REPO_ROOT/bench.py --global-batch 32 --steps 20 --warmup 5 --ref-window 0 > $D.log 2>&1) || { tail -5 $D.log; exit 1; }
  echo profiled
fi
