#!/bin/bash
# Two-bucket overlap study (stand-in collectives): the big early bucket (512-channel layers)
# on the comm stream overlapping the rest of the backward, vs everything inline.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
b() { local label=$1 envs=$2; shift 2
  timeout -k 10 200 env $envs python bench.py --steps 60 --warmup 10 "$@" > gpurun_out/ov.log 2>&1 || { tail -5 gpurun_out/ov.log; exit 1; }
  echo "| $label | $envs $* | $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ov.log | cut -d' ' -f2) |"; }
for i in 1 2; do
b inline_1bucket "DDP_AMD_EMULATE_COMM=1"
b inline_2buckets "DDP_AMD_EMULATE_COMM=1" --first-bucket-mb 34 --bucket-mb 64
b stream_2buckets "DDP_AMD_EMULATE_COMM=1 DDP_AMD_COMM_OVERLAP=1" --first-bucket-mb 34 --bucket-mb 64
b stream_2buckets_eager "DDP_AMD_EMULATE_COMM=1 DDP_AMD_COMM_OVERLAP=1" --first-bucket-mb 34 --bucket-mb 64 --no-graph
b inline_2buckets_eager "DDP_AMD_EMULATE_COMM=1" --first-bucket-mb 34 --bucket-mb 64 --no-graph
done
