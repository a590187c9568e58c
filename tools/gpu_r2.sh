#!/bin/bash
# Round-2 check: GPU tests, default bench (global 256), the 8-GPU strong-scaling share (b32),
# and a rocprofv3 kernel trace of the b32 step.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/r2
TESTS=${TESTS:-tests}
timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r2/gputests.log 2>&1 || { tail -40 gpurun_out/r2/gputests.log; exit 1; }
tail -2 gpurun_out/r2/gputests.log
timeout -k 10 200 python bench.py > gpurun_out/r2/bench_default.log 2>&1 || { tail -5 gpurun_out/r2/bench_default.log; exit 1; }
tail -1 gpurun_out/r2/bench_default.log
timeout -k 10 200 python bench.py --global-batch 32 > gpurun_out/r2/bench_b32.log 2>&1 || { tail -5 gpurun_out/r2/bench_b32.log; exit 1; }
tail -1 gpurun_out/r2/bench_b32.log
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r2/prof_b32" -o vgg11 -- python3 "$GRAFT_REPO_ROOT/bench.py" --global-batch 32 --steps 20 --warmup 5 --ref-window 0 > "$GRAFT_REPO_ROOT/gpurun_out/r2/prof_b32.log" 2>&1) || { tail -5 gpurun_out/r2/prof_b32.log; exit 1; }
echo profiled
