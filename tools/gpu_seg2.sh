#!/bin/bash
# Segmented step (three graphs, late bucket on a second stream) vs single graph, timed 32-CU
# stand-in collectives at modelled all-reduce bandwidths (GB/s).
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
b() { local label=$1 envs=$2; shift 2
  timeout -k 10 200 env $envs python bench.py --steps 60 --warmup 10 "$@" > gpurun_out/seg.log 2>&1 || { tail -5 gpurun_out/seg.log; exit 1; }
  echo "| $label | $envs $* | $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/seg.log | cut -d' ' -f2) |"; }
echo "| variant | settings | ms/step |"
echo "|---|---|---|"
for i in 1 2; do
b base "DDP_AMD_EMULATE_COMM=0"
b seg4_nocomm "DDP_AMD_EMULATE_COMM=0" --segmented 4
b seg4_nocomm_events "DDP_AMD_SEG_MODE=events" --segmented 4
for g in 300 171 100; do
b inline_$g "DDP_AMD_EMULATE_COMM_GBPS=$g"
b seg4_$g "DDP_AMD_EMULATE_COMM_GBPS=$g" --segmented 4
b seg4_events_$g "DDP_AMD_SEG_MODE=events DDP_AMD_EMULATE_COMM_GBPS=$g" --segmented 4
done
done
