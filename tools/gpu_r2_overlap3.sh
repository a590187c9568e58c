#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/ovl3
for M in eager pipelined; do for B in 32 256; do
  DDP_AMD_RCCL_SELF=1 timeout -k 10 120 python tools/overlap_probe.py --mode $M --batch $B > gpurun_out/ovl3/${M}_b$B.md 2>&1 || { tail -20 gpurun_out/ovl3/${M}_b$B.md; exit 1; }
  tail -1 gpurun_out/ovl3/${M}_b$B.md | cut -c1-300
done; done
DDP_AMD_RCCL_SELF=1 GPU_MAX_HW_QUEUES=8 timeout -k 10 120 python tools/overlap_probe.py --mode pipelined --batch 32 > gpurun_out/ovl3/pipelined_b32_q8.md 2>&1 || exit 1
tail -1 gpurun_out/ovl3/pipelined_b32_q8.md | cut -c1-300
for B in 32 256; do
  for V in seg0 seg; do
    S="--segmented 0"; [ $V = seg ] && S=""
    [ $V = seg ] && S="--segmented $([ $B = 32 ] && echo 3,6 || echo 2,5)"
    DDP_AMD_EMULATE_COMM_GBPS=171 timeout -k 10 120 python bench.py --global-batch $B --steps 60 --warmup 10 --ref-window 0 $S > gpurun_out/ovl3/bench_emu_${V}_b$B.log 2>&1 || exit 1
    DDP_AMD_RCCL_SELF=1 timeout -k 10 120 python bench.py --global-batch $B --steps 60 --warmup 10 --ref-window 0 $S > gpurun_out/ovl3/bench_rccl_${V}_b$B.log 2>&1 || exit 1
    echo "B=$B $V emu $(tail -1 gpurun_out/ovl3/bench_emu_${V}_b$B.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])') rccl $(tail -1 gpurun_out/ovl3/bench_rccl_${V}_b$B.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
  done
done
