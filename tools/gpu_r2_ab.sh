#!/bin/bash
# A/B of the launch-reduction changes (split-K ticket fixup, WGRAD atomics, BN-backward finalize
# fold) at the strong-scaling batches, plus the per-dispatch floor microbenchmark.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/kernels.log 2>&1 || { tail -30 gpurun_out/ab/kernels.log; exit 1; }
tail -1 gpurun_out/ab/kernels.log
timeout -k 10 120 python tools/launch_floor.py > gpurun_out/ab/floor_default.log 2>&1 || { tail gpurun_out/ab/floor_default.log; exit 1; }
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 120 python tools/launch_floor.py > gpurun_out/ab/floor_nocapture.log 2>&1 || { tail gpurun_out/ab/floor_nocapture.log; exit 1; }
for B in 32 64 128 256; do
  for V in base fixup all; do
    case $V in
      base) E="DDP_AMD_FIXUP=0 DDP_AMD_WGRAD_ATOMIC=0 DDP_AMD_BN_FOLD_BWD_KB=0";;
      fixup) E="DDP_AMD_BN_FOLD_BWD_KB=0";;
      all) E="";;
    esac
    env $E timeout -k 10 120 python bench.py --global-batch $B --steps 60 --warmup 10 --ref-window 0 > gpurun_out/ab/b${B}_$V.log 2>&1 || { tail -5 gpurun_out/ab/b${B}_$V.log; exit 1; }
    echo "B=$B $V $(python -c "import json,sys; d=json.loads(open('gpurun_out/ab/b${B}_$V.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['train_loss_mean'])")"
  done
done
