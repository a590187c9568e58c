#!/bin/bash
# Split-K finish passes with batched slab loads: conv numerics tests, then a same-session A/B of
# the previous build (ab_so/_native_old.so) vs this build at 2 and 1 rows per thread
# (DDP_AMD_FINISH_RPT), VGG-11 b256 / b32 and ResNet-50 b256, two interleaved passes.
cd "$GRAFT_REPO_ROOT" || exit 2
OUT=gpurun_out/finish
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
CFGS=${CFGS:-"vgg11:256 vgg11:32 resnet50:256"}
for P in 1 2; do
  for CFG in $CFGS; do
    M=${CFG%%:*}; B=${CFG##*:}; S=60; [ $M = resnet50 ] && S=20
    for V in old rpt2 rpt1; do
      L=$OUT/${M}_b${B}_${V}_p$P.log
      NP=""; RPT=2
      [ $V = old ] && NP=ab_so/_native_old.so
      [ $V = rpt1 ] && RPT=1
      DDP_AMD_NATIVE_PATH=$NP DDP_AMD_FINISH_RPT=$RPT timeout -k 10 240 python bench.py --model $M --global-batch $B --steps $S --warmup 10 --ref-window 0 > $L 2>&1 || { tail -5 $L; exit 1; }
      echo "$M B=$B $V p$P $(python -c "import json; d=json.loads(open('$L').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['train_loss_mean'])")"
    done
  done
done
if [ -n "$PROF" ]; then
  D=$GRAFT_REPO_ROOT/$OUT/prof_b32
  (cd /tmp && export TMPDIR=/tmp && DDP_AMD_FINISH_RPT=${PROF_RPT:-1} timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o p -- python3 $GRAFT_REPO_ROOT/bench.py --global-batch 32 --steps 20 --warmup 5 --ref-window 0 > $D.log 2>&1) || { tail -5 $D.log; exit 1; }
  echo profiled
fi
