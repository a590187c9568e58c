#!/bin/bash
# round 5: full GPU suite, then the pipelined-step probes and the stand-in sweep (corrected stand-in)
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r5c; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { grep -E "FAIL|Error" $O/gpu_tests.log | head -20; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for cfg in "32 3,6 shard16" "32 3,6 allreduce" "32 3,5,7 allreduce"; do
  set -- $cfg
  timeout -k 10 120 python tools/pipeline_probe.py --batch $1 --cuts $2 --update $3 > $O/probe_b$1_${2//,/-}_$3.md 2>&1 || { tail -20 $O/probe_b$1_${2//,/-}_$3.md; exit 1; }
  grep -E "^\| (standin|nocomm)|contention" $O/probe_b$1_${2//,/-}_$3.md
done
TAG=r5c_sweep BATCHES="32 64 128 256" CUTS="3,6 3,5,7 4 2,5" PASSES=1 bash tools/gpu/standin_sweep.sh
