#!/bin/bash
# Same-session A/B of environment settings: GPU kernel + model tests, then bench.py for every
# variant x config, two interleaved passes; optional rocprofv3 table of the last variant at b32.
#   VARIANTS="base: r512:DDP_AMD_BN_BWD_FUSE_MAX_ROWS=512" CFGS="vgg11:32 vgg11:256" bash tools/gpu/ab_env.sh
cd "$GRAFT_REPO_ROOT" || exit 2
OUT=gpurun_out/abenv
mkdir -p $OUT
if [ -z "$NOTEST" ]; then
  timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
  tail -1 $OUT/tests.log
fi
CFGS=${CFGS:-"vgg11:32 vgg11:64 vgg11:128 vgg11:256"}
for P in 1 2; do
  for CFG in $CFGS; do
    M=${CFG%%:*}; B=${CFG##*:}; S=60; [ $M = resnet50 ] && S=20
    for V in $VARIANTS; do
      NAME=${V%%:*}; ENVS=${V#*:}
      L=$OUT/${M}_b${B}_${NAME}_p$P.log
      env ${ENVS//,/ } timeout -k 10 240 python bench.py --model $M --global-batch $B --steps $S --warmup 10 --ref-window 0 > $L 2>&1 || { tail -5 $L; exit 1; }
      echo "$M B=$B $NAME p$P $(python -c "import json; d=json.loads(open('$L').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['train_loss_mean'])")"
    done
  done
done
if [ -n "$PROF" ]; then
  V=${VARIANTS##* }; ENVS=${V#*:}
  D=$GRAFT_REPO_ROOT/$OUT/prof_b32
  (cd /tmp && export TMPDIR=/tmp && export ${ENVS//,/ } && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o p -- python3 $GRAFT_REPO_ROOT/bench.py --global-batch 32 --steps 20 --warmup 5 --ref-window 0 > $D.log 2>&1) || { tail -5 $D.log; exit 1; }
  echo profiled
fi
