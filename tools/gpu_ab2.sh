#!/bin/bash
# same-box A/B of two env settings, interleaved: bash tools/gpu_ab2.sh "ENV_A" "ENV_B" [reps]
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
A=$1; B=$2; n=${3:-3}
for i in $(seq 1 $n); do
  for lab in A B; do
    envs=$A; [ $lab = B ] && envs=$B
    timeout -k 10 200 env $envs python bench.py --steps 60 --warmup 10 > gpurun_out/ab2.log 2>&1 || { tail -3 gpurun_out/ab2.log; exit 1; }
    echo "$lab [$envs] $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab2.log)"
  done
done
