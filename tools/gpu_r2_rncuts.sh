#!/bin/bash
# ResNet-50 b256: pipelined DDP step cut points with the 171 GB/s stand-in collective
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/rncuts
for C in 0 8,14 4,8,14 14; do
  DDP_AMD_EMULATE_COMM_GBPS=171 timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 3 --ref-window 0 --segmented $C > gpurun_out/rncuts/c${C//,/-}.log 2>&1 || { tail -5 gpurun_out/rncuts/c${C//,/-}.log; exit 1; }
  echo "cuts=$C $(tail -1 gpurun_out/rncuts/c${C//,/-}.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
done
timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 3 --ref-window 0 > gpurun_out/rncuts/none.log 2>&1 || exit 1
echo "no collective $(tail -1 gpurun_out/rncuts/none.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
