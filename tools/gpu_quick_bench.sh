#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/qb
timeout -k 10 120 python bench.py --steps 100 --warmup 10 --ref-window 0 > gpurun_out/qb/b256.log 2>&1 || exit 1
echo "b256 $(tail -1 gpurun_out/qb/b256.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
timeout -k 10 120 python bench.py --global-batch 32 --steps 100 --warmup 10 --ref-window 0 > gpurun_out/qb/b32.log 2>&1 || exit 1
echo "b32 $(tail -1 gpurun_out/qb/b32.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 3 --ref-window 0 > gpurun_out/qb/rn.log 2>&1 || exit 1
echo "resnet $(tail -1 gpurun_out/qb/rn.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
rocm-smi --showclocks 2>/dev/null | grep -i "sclk\|mclk" | head -4 || true
