#!/bin/bash
# kernel + model GPU tests, then the three headline benches (and a b32 kernel-stats profile)
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/q
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_resnet.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/q/tests.log 2>&1 || { tail -30 gpurun_out/q/tests.log; exit 1; }
tail -1 gpurun_out/q/tests.log
for CFG in "vgg11 256" "vgg11 32" "resnet50 256"; do
  set -- $CFG; M=$1; B=$2; S=60; [ $M = resnet50 ] && S=20
  L=gpurun_out/q/${M}_b$B.log
  timeout -k 10 240 python bench.py --model $M --global-batch $B --steps $S --warmup 10 --ref-window 0 > $L 2>&1 || { tail -5 $L; exit 1; }
  echo "$M B=$B $(python -c "import json; d=json.loads(open('$L').read().strip().splitlines()[-1]); print(d['ms_per_step'], d.get('train_loss_mean'))")"
done
if [ -n "$PROF" ]; then
  D=$GRAFT_REPO_ROOT/gpurun_out/q/prof_b32
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o p -- python3 $GRAFT_REPO_ROOT/bench.py --global-batch 32 --steps 20 --warmup 5 --ref-window 0 > $D.log 2>&1) || { tail -5 $D.log; exit 1; }
  echo profiled
fi
