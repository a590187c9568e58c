#!/bin/bash
# round 5: cut-planner ground truth on the round-5 kernels: stage times at b32/64/128/256, then
# the stand-in sweep (allreduce vs shard16 vs mixed) over the cut sets of tests/test_cut_plan.py
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r5d; mkdir -p $O
for B in 32 64 128 256; do
  timeout -k 10 120 python tools/stage_times.py --batch $B > $O/stages_b$B.json 2> $O/stages_b$B.err || { tail -5 $O/stages_b$B.err; exit 1; }
  cat $O/stages_b$B.json
done
TAG=r5d_sweep BATCHES="32 256" CUTS="3,6 3,5,7 4 2,5 2,4,6 4,6 5" PASSES=1 bash tools/gpu/standin_sweep.sh || exit 1
TAG=r5d_sweep2 BATCHES="64 128" CUTS="3,6 3,5,7 2,5 4" PASSES=1 bash tools/gpu/standin_sweep.sh || exit 1
TAG=r5d_mixed BATCHES="32 64 128" CUTS="3,6" UPDATES="s16,s16,ar s16,ar,ar auto" PASSES=1 bash tools/gpu/standin_sweep.sh
