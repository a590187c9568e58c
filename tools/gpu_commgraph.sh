#!/bin/bash
# One-GPU study of the multi-GPU step graph: DDP with stand-in collectives (DDP_AMD_EMULATE_COMM=1:
# one bucket-sized pass per collective) inline on the step stream vs on a comm stream.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
b() {  # label "ENV=.. ENV=.." bench-args...
  local label=$1 envs=$2; shift 2
  timeout -k 10 200 env $envs python bench.py --steps 40 --warmup 10 "$@" > "gpurun_out/cg_$label.log" 2>&1 || { tail -5 "gpurun_out/cg_$label.log"; exit 1; }
  echo "| $label | $envs $* | $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/cg_$label.log | cut -d' ' -f2) |"
}
echo "| variant | settings | ms/step |"
echo "|---|---|---|"
b base "DDP_AMD_EMULATE_COMM=0"
b inline_1bucket "DDP_AMD_EMULATE_COMM=1"
b inline_8mb "DDP_AMD_EMULATE_COMM=1" --bucket-mb 8 --first-bucket-mb 1
b stream_8mb "DDP_AMD_EMULATE_COMM=1 DDP_AMD_COMM_OVERLAP=1" --bucket-mb 8 --first-bucket-mb 1
b stream_1bucket "DDP_AMD_EMULATE_COMM=1 DDP_AMD_COMM_OVERLAP=1"
b eager_inline_8mb "DDP_AMD_EMULATE_COMM=1" --bucket-mb 8 --first-bucket-mb 1 --no-graph
b eager_stream_8mb "DDP_AMD_EMULATE_COMM=1 DDP_AMD_COMM_OVERLAP=1" --bucket-mb 8 --first-bucket-mb 1 --no-graph
exit 0
