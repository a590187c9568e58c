#!/bin/bash
# No-pool BN-backward sums in the lean dgrad epilogue (BNF 2): numerics, then ResNet-50 b256
# with DDP_AMD_BN_BWD_FUSE_NOPOOL=0/1 for the in-tree build and the base build, and VGG checks
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/bnf
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_resnet.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/bnf/tests.log 2>&1 || { tail -30 gpurun_out/bnf/tests.log; exit 1; }
tail -1 gpurun_out/bnf/tests.log
DDP_AMD_BN_BWD_FUSE_NOPOOL=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_resnet.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/bnf/tests_np.log 2>&1 || { tail -30 gpurun_out/bnf/tests_np.log; exit 1; }
tail -1 gpurun_out/bnf/tests_np.log
for P in 1 2; do
  for V in base cur; do
    for NP in 0 1; do
      if [ $V = base ]; then NPATH=ab_so/_native_base.so; else NPATH=""; fi
      L=gpurun_out/bnf/rn_${V}_np${NP}_p$P.log
      DDP_AMD_NATIVE_PATH=$NPATH DDP_AMD_BN_BWD_FUSE_NOPOOL=$NP timeout -k 10 200 python bench.py --model resnet50 --steps 20 --warmup 8 --ref-window 0 > $L 2>&1 || { tail -5 $L; exit 1; }
      echo "resnet50 $V nopool=$NP p$P $(python -c "import json; d=json.loads(open('$L').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['train_loss_mean'])")"
    done
  done
  for V in base cur; do
    if [ $V = base ]; then NPATH=ab_so/_native_base.so; else NPATH=""; fi
    for B in 256 32; do
      L=gpurun_out/bnf/vgg_b${B}_${V}_p$P.log
      DDP_AMD_NATIVE_PATH=$NPATH timeout -k 10 120 python bench.py --global-batch $B --steps 60 --warmup 10 --ref-window 0 > $L 2>&1 || { tail -5 $L; exit 1; }
      echo "vgg11 B=$B $V p$P $(python -c "import json; d=json.loads(open('$L').read().strip().splitlines()[-1]); print(d['ms_per_step'])")"
    done
  done
done
