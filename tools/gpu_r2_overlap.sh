#!/bin/bash
# device-side (HIP timing events) timelines of the eager and pipelined DDP steps with live
# single-rank RCCL collectives, plus a kernel trace of the eager one
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/ovl
for M in eager pipelined; do
  for B in 32 256; do
    DDP_AMD_RCCL_SELF=1 timeout -k 10 180 python tools/overlap_probe.py --mode $M --batch $B > gpurun_out/ovl/probe_${M}_b$B.md 2>&1 || { tail -20 gpurun_out/ovl/probe_${M}_b$B.md; exit 1; }
    tail -1 gpurun_out/ovl/probe_${M}_b$B.md | cut -c1-400
  done
done
