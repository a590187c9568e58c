#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
root="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 -L > "$root/gpurun_out/counters_list.txt" 2>&1)
echo "list rc=$?"
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats \
    --output-format csv -d "$root/gpurun_out/prof_resnet" -o resnet -- \
    python3 "$root/bench.py" --model resnet50 --steps 6 --warmup 3 > "$root/gpurun_out/prof_resnet.log" 2>&1)
rc=$?; tail -2 gpurun_out/prof_resnet.log; echo "prof rc=$rc"
exit $rc
