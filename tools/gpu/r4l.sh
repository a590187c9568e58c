#!/bin/bash
# round 4: full GPU test suite on the L0 v5 build, then the default bench line
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r4l; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { grep -E "FAIL|Error" $O/gpu_tests.log | head -20; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 200 python bench.py > $O/bench_default.log 2>&1 || { tail -5 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log
