#!/bin/bash
# Segmented step v3 (two graphs, event fork, device-side wait before the optimizer) vs inline.
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
for g in 300 171 100; do
b inline_$g "DDP_AMD_EMULATE_COMM_GBPS=$g"
b seg4_$g "DDP_AMD_EMULATE_COMM_GBPS=$g" --segmented 4
b seg3_$g "DDP_AMD_EMULATE_COMM_GBPS=$g" --segmented 3
done
done
mkdir -p gpurun_out/prof_seg
DDP_AMD_EMULATE_COMM_GBPS=171 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_seg -o seg4v3 -- python bench.py --steps 20 --warmup 5 --segmented 4 > gpurun_out/prof_seg.log 2>&1 || { tail -5 gpurun_out/prof_seg.log; exit 1; }
echo profiled
