#!/bin/bash
# Round-2 full check: every GPU test, smoke(), default bench (N=1 headline), b32 bench
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/full
timeout -k 10 900 python -u -m pytest tests -m gpu ${GPU_TEST_SEL:-} -x -v --timeout 300 --timeout-method thread > gpurun_out/full/gputests.log 2>&1 || { tail -40 gpurun_out/full/gputests.log; exit 1; }
tail -1 gpurun_out/full/gputests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/full/smoke.log 2>&1 || { tail -20 gpurun_out/full/smoke.log; exit 1; }
tail -1 gpurun_out/full/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/full/bench.log 2>&1 || { tail -5 gpurun_out/full/bench.log; exit 1; }
tail -1 gpurun_out/full/bench.log
timeout -k 10 300 python bench.py --global-batch 32 > gpurun_out/full/bench_b32.log 2>&1 || { tail -5 gpurun_out/full/bench_b32.log; exit 1; }
tail -1 gpurun_out/full/bench_b32.log | cut -c1-200
