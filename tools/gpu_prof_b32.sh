#!/bin/bash
# rocprofv3 kernel trace of the b32 step under a given env (arg 1 = tag, rest = env assignments)
cd "$GRAFT_REPO_ROOT" || exit 2
TAG=$1; shift
mkdir -p gpurun_out/pb
(cd /tmp && export TMPDIR=/tmp && env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pb/$TAG" -o vgg11 -- python3 "$GRAFT_REPO_ROOT/bench.py" --global-batch ${B:-32} --steps 20 --warmup 5 --ref-window 0 > "$GRAFT_REPO_ROOT/gpurun_out/pb/$TAG.log" 2>&1) || { tail -5 gpurun_out/pb/$TAG.log; exit 1; }
tail -1 gpurun_out/pb/$TAG.log | cut -c1-200
