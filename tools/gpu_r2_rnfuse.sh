#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/rnf
timeout -k 10 400 python -u -m pytest tests/test_gpu_resnet.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/rnf/tests.log 2>&1 || { tail -30 gpurun_out/rnf/tests.log; exit 1; }
tail -1 gpurun_out/rnf/tests.log
for V in 0 1; do
  DDP_AMD_BN_BWD_FUSE_NOPOOL=$V timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 3 --ref-window 0 > gpurun_out/rnf/b$V.log 2>&1 || { tail -5 gpurun_out/rnf/b$V.log; exit 1; }
  echo "nopool_fuse=$V $(tail -1 gpurun_out/rnf/b$V.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["train_loss_mean"])')"
done
