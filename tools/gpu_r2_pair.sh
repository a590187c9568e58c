#!/bin/bash
# backward pair kernel: kernel tests, model tests, bench A/B (pair 0/1/2) at b32..b256
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/pair
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "pair or dgrad or splitk" > gpurun_out/pair/kernels.log 2>&1 || { tail -30 gpurun_out/pair/kernels.log; exit 1; }
tail -1 gpurun_out/pair/kernels.log
for M in 3 2; do
  DDP_AMD_BWD_PAIR=$M timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -m gpu -x -q --timeout 200 --timeout-method thread -k "oracle and not trajectory" > gpurun_out/pair/model_$M.log 2>&1 || { tail -30 gpurun_out/pair/model_$M.log; exit 1; }
  echo "model pair=$M $(tail -1 gpurun_out/pair/model_$M.log)"
done
for B in 32 64 128 256; do
  for M in 0 1 3; do
    DDP_AMD_BWD_PAIR=$M timeout -k 10 120 python bench.py --global-batch $B --steps 60 --warmup 10 --ref-window 0 > gpurun_out/pair/b${B}_$M.log 2>&1 || { tail -5 gpurun_out/pair/b${B}_$M.log; exit 1; }
    echo "B=$B pair=$M $(tail -1 gpurun_out/pair/b${B}_$M.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["train_loss_mean"])')"
  done
done
