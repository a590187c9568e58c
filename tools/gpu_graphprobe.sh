#!/bin/bash
# hipGraph branch-cost probe under several runtime settings
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
run() { echo "== $*"; timeout -k 10 120 "$@" || exit $?; }
run python tools/graph_branch_probe.py
run env DEBUG_HIP_FORCE_GRAPH_QUEUES=1 python tools/graph_branch_probe.py
run env DEBUG_HIP_FORCE_GRAPH_QUEUES=2 python tools/graph_branch_probe.py
run env DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 python tools/graph_branch_probe.py
run env DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 python tools/graph_branch_probe.py
run python tools/graph_branch_probe.py --every 40
echo "== eager bench side on/off"
DDP_AMD_BWD_STREAMS=1 timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-graph | grep -o '"ms_per_step": [0-9.]*' || exit 1
DDP_AMD_BWD_STREAMS=0 timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-graph | grep -o '"ms_per_step": [0-9.]*' || exit 1
echo "== graph bench side on, FORCE_GRAPH_QUEUES=1"
DEBUG_HIP_FORCE_GRAPH_QUEUES=1 DDP_AMD_BWD_STREAMS=1 timeout -k 10 200 python bench.py --steps 30 --warmup 5 | grep -o '"ms_per_step": [0-9.]*' || exit 1
exit 0
