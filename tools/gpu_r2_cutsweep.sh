#!/bin/bash
# Cut-point sweep of the pipelined DDP step (VGG-11) at the strong-scaling per-GPU batches,
# with the timed 32-CU stand-in collective at G GB/s algorithm bandwidth.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/cuts
for G in 171 300; do
for B in 32 64 128 256; do
  for C in 0 4 3,6 2,5 2,4,6 3,5,7 1,3,5 3,5 4,6 2,6; do
    tag=b${B}_g${G}_c${C//,/-}
    DDP_AMD_EMULATE_COMM_GBPS=$G timeout -k 10 120 python bench.py --global-batch $B --steps 60 --warmup 10 --ref-window 0 --segmented $C > gpurun_out/cuts/$tag.log 2>&1 || { tail -5 gpurun_out/cuts/$tag.log; exit 1; }
    echo "$B $G $C $(python -c "import json; d=json.loads(open('gpurun_out/cuts/$tag.log').read().strip().splitlines()[-1]); print(d['ms_per_step'])")"
  done
  [ "$G" = 300 ] && [ "$B" = 64 ] && break
done
done
