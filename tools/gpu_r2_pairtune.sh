#!/bin/bash
# Backward-pair split-K tuning (mode-3 table entries), then bench A/B against the shipped table
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/pt
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "pair" --timeout 120 --timeout-method thread > gpurun_out/pt/tests.log 2>&1 || { tail -30 gpurun_out/pt/tests.log; exit 1; }
tail -1 gpurun_out/pt/tests.log
timeout -k 10 600 python -u tools/conv_tune.py --pairs --reps 20 --out gpurun_out/pt/conv_tuning_pairs.json > gpurun_out/pt/tune.log 2>&1 || { tail -20 gpurun_out/pt/tune.log; exit 1; }
cat gpurun_out/pt/tune.log
for P in 1 2; do
for B in 32 64 128 256; do
  for T in base pairs; do
    case $T in base) F=distributed-data-parallel-ml-training_amd/ops/conv_tuning.json;; *) F=gpurun_out/pt/conv_tuning_pairs.json;; esac
    L=gpurun_out/pt/b${B}_${T}_p$P.log
    DDP_AMD_CONV_TUNING_FILE=$F timeout -k 10 120 python bench.py --global-batch $B --steps 60 --warmup 10 --ref-window 0 > $L 2>&1 || { tail -5 $L; exit 1; }
    echo "B=$B $T p$P $(python -c "import json; d=json.loads(open('$L').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['train_loss_mean'])")"
  done
done
done
