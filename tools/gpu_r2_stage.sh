#!/bin/bash
# LDS-staged 16-B output stores in the conv GEMM epilogue: numerics + A/B
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/stage
DDP_AMD_STAGE_OUT=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "conv" > gpurun_out/stage/kernels.log 2>&1 || { tail -30 gpurun_out/stage/kernels.log; exit 1; }
tail -1 gpurun_out/stage/kernels.log
DDP_AMD_STAGE_OUT=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -m gpu -x -q --timeout 200 --timeout-method thread -k "oracle and not trajectory" > gpurun_out/stage/model.log 2>&1 || { tail -30 gpurun_out/stage/model.log; exit 1; }
tail -1 gpurun_out/stage/model.log
for B in 256 32; do
  for rep in 1 2; do
    for V in 0 1; do
      DDP_AMD_STAGE_OUT=$V timeout -k 10 120 python bench.py --global-batch $B --steps 100 --warmup 10 --ref-window 0 > gpurun_out/stage/b${B}_$V.log 2>&1 || { tail -5 gpurun_out/stage/b${B}_$V.log; exit 1; }
      echo "B=$B stage=$V rep=$rep $(tail -1 gpurun_out/stage/b${B}_$V.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
    done
  done
done
for V in 0 1; do
  DDP_AMD_STAGE_OUT=$V timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 3 --ref-window 0 > gpurun_out/stage/rn_$V.log 2>&1 || exit 1
  echo "resnet stage=$V $(tail -1 gpurun_out/stage/rn_$V.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
done
