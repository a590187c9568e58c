#!/bin/bash
# Backward-pair tuning for ResNet-50 b256 stride-1 layers, merged into the shipped table; A/B
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/ptr
timeout -k 10 900 python -u tools/conv_tune.py --pairs --pair-sets "resnet50:256" --reps 10 --merge distributed-data-parallel-ml-training_amd/ops/conv_tuning.json --out gpurun_out/ptr/conv_tuning_rn.json > gpurun_out/ptr/tune.log 2>&1 || { tail -20 gpurun_out/ptr/tune.log; exit 1; }
cat gpurun_out/ptr/tune.log
for P in 1 2; do
  for T in base rn; do
    case $T in base) F=distributed-data-parallel-ml-training_amd/ops/conv_tuning.json;; *) F=gpurun_out/ptr/conv_tuning_rn.json;; esac
    L=gpurun_out/ptr/rn_${T}_p$P.log
    DDP_AMD_CONV_TUNING_FILE=$F timeout -k 10 200 python bench.py --model resnet50 --steps 20 --warmup 8 --ref-window 0 > $L 2>&1 || { tail -5 $L; exit 1; }
    echo "resnet50 $T p$P $(python -c "import json; d=json.loads(open('$L').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['train_loss_mean'])")"
  done
done
