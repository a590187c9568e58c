#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
timeout -k 10 100 python tools/graph_branch_probe.py --join-end || exit 1
timeout -k 10 100 python tools/graph_branch_probe.py --join-end --every 20 || exit 1
for ov in 1 0; do
  DDP_AMD_EMULATE_COMM=1 DDP_AMD_COMM_OVERLAP=$ov timeout -k 10 200 python bench.py --steps 40 --warmup 10 --no-graph > gpurun_out/eager_$ov.log 2>&1 || exit 1
  echo "eager overlap=$ov $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/eager_$ov.log)"
done
exit 0
