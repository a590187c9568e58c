#!/bin/bash
# round 4 final: per-GPU-share step times of the shipped build (b256/b128/b64/b32, 2 passes),
# ResNet-50 b256 step + profile
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r4v; mkdir -p $O
for P in 1 2; do
for CFG in 256 128 64 32; do
  L=$O/b${CFG}_p$P.log
  timeout -k 10 200 python bench.py --global-batch $CFG --steps 60 --warmup 10 --ref-window 0 > $L 2>&1 || { tail -5 $L; exit 1; }
  echo "b$CFG p$P $(python -c "import json; d=json.loads(open('$L').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'])")"
done
done
L=$O/resnet.log
timeout -k 10 300 python bench.py --model resnet50 --steps 8 --warmup 4 --ref-window 0 > $L 2>&1 || { tail -5 $L; exit 1; }
echo "resnet50 $(python -c "import json; d=json.loads(open('$L').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'])")"
TAG=r4v MODEL=resnet50 BATCHES="256" bash tools/gpu/profile.sh || exit 1
TAG=r4v BATCHES="128 64" bash tools/gpu/profile.sh || exit 1
