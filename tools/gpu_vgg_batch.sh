#!/bin/bash
# VGG-11 step time vs per-GPU batch (the strong-scaling split of global batch 256 over 1/2/4/8 GPUs)
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
for b in 32 64 128 256; do
  timeout -k 10 200 python bench.py --per-gpu-batch $b --steps 60 --warmup 10 > gpurun_out/vb_$b.log 2>&1 || { tail -3 gpurun_out/vb_$b.log; exit 1; }
  echo "B=$b $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/vb_$b.log) $(grep -o '"value": [0-9.]*' gpurun_out/vb_$b.log)"
done
root="$GRAFT_REPO_ROOT"
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
   -d "$root/gpurun_out/prof_b32" -o vgg32 -- python3 "$root/bench.py" --per-gpu-batch 32 --steps 10 --warmup 3 \
   > "$root/gpurun_out/prof_b32.log" 2>&1) || exit 1
