#!/bin/bash
# round 5: sharded bf16-gather update — GPU tests of the new paths, then the stand-in sweep
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r5a; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_rccl_self.py tests/test_gpu_model.py -k "shard16 or live_rccl or segmented" > $O/tests.log 2>&1 \
  || { grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
grep -E "PASS|FAIL" $O/tests.log | tail -20; tail -1 $O/tests.log
TAG=r5a_sweep BATCHES="32 64 128" CUTS="3,6 3,5,7" PASSES=1 bash tools/gpu/standin_sweep.sh
