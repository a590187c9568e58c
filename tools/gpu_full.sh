#!/bin/bash
# Round-end rehearsal: full GPU test suite, smoke(), default bench, rocprofv3 stats of the bench.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/prof_full
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { tail -30 gpurun_out/gputests.log; exit 1; }
tail -2 gpurun_out/gputests.log
timeout -k 10 200 python -c 'import __graft_entry__ as g; g.smoke()' || exit 1
timeout -k 10 200 python bench.py > gpurun_out/bench_default.log 2>&1 || { tail -5 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_full" -o vgg11 -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 > "$GRAFT_REPO_ROOT/gpurun_out/prof_full.log" 2>&1) || { tail -5 gpurun_out/prof_full.log; exit 1; }
echo profiled
