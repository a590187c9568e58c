#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
timeout -k 10 100 python tools/graph_branch_probe.py || exit 1
timeout -k 10 100 python tools/graph_branch_probe.py --segmented || exit 1
timeout -k 10 100 python tools/graph_branch_probe.py --segmented --nk 160 || exit 1
exit 0
