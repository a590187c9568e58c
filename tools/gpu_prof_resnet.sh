#!/bin/bash
# ResNet-50 b256 bench + rocprofv3 kernel trace of a few steps
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/rn
timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 3 --ref-window 0 > gpurun_out/rn/bench.log 2>&1 || { tail -5 gpurun_out/rn/bench.log; exit 1; }
tail -1 gpurun_out/rn/bench.log | cut -c1-300
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/rn/prof" -o rn -- python3 "$GRAFT_REPO_ROOT/bench.py" --model resnet50 --steps 4 --warmup 3 --ref-window 0 > "$GRAFT_REPO_ROOT/gpurun_out/rn/prof.log" 2>&1) || { tail -5 gpurun_out/rn/prof.log; exit 1; }
echo profiled
