#!/bin/bash
# every bench.py variant runs (1 GPU): strategies, eager, strong-scaling flag, ResNet, bf16 comm
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
run() { local label=$1; shift; timeout -k 10 200 python bench.py --steps 20 --warmup 5 "$@" > gpurun_out/bv.log 2>&1 || { echo "$label FAILED"; tail -5 gpurun_out/bv.log; exit 1; }; echo "$label $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bv.log) $(grep -o '"hipgraph": [a-z]*' gpurun_out/bv.log)"; }
run ddp
run allreduce --strategy allreduce
run gather_scatter --strategy gather_scatter
run gather_broadcast --strategy gather_broadcast
run eager --no-graph
run strong256 --global-batch 256
run bf16comm --grad-comm bf16
run reference_buckets --bucket-mb 25 --first-bucket-mb 1
run vgg16 --model vgg16
run resnet64 --model resnet50 --per-gpu-batch 64
