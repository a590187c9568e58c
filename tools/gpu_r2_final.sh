#!/bin/bash
# Round-end rehearsal: every GPU test, smoke(), the default bench (N=1 headline) and the b32
# share, then rocprofv3 kernel tables of the b256 and b32 steps.
cd "$GRAFT_REPO_ROOT" || exit 2
bash tools/gpu_r2_full.sh || exit 1
for B in 256 32; do
  D=$GRAFT_REPO_ROOT/gpurun_out/final/prof_b$B
  mkdir -p $GRAFT_REPO_ROOT/gpurun_out/final
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o p -- python3 $GRAFT_REPO_ROOT/bench.py --global-batch $B --steps 20 --warmup 5 --ref-window 0 > $D.log 2>&1) || { tail -5 $D.log; exit 1; }
done
echo profiled
