#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/prof_fx
(cd /tmp && export TMPDIR=/tmp && DDP_AMD_SPLITK_FIXUP=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_fx" -o fx -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 3 > "$GRAFT_REPO_ROOT/gpurun_out/prof_fx.log" 2>&1) || { tail -5 gpurun_out/prof_fx.log; exit 1; }
echo ok
