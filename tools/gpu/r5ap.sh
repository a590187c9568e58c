#!/bin/bash
# round 5: ResNet stem conv (conv_smallk_lds_kernel) in 512-thread blocks — stem / smallk kernel
# tests, ResNet-50 b256 A/B (DDP_AMD_STEM_THREADS=256 vs 512, interleaved), kernel profile
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r5ap; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_resnet.py -k "conv_fwd_stats or resnet50_train_step or bottleneck" -x -q --timeout 300 --timeout-method thread > $O/tests_k.log 2>&1 || { tail -30 $O/tests_k.log; exit 1; }
tail -1 $O/tests_k.log
for i in 1 2; do
  for t in 256 512; do
    DDP_AMD_STEM_THREADS=$t timeout -k 10 300 python bench.py --model resnet50 --steps 8 --warmup 4 --ref-window 0 > $O/resnet_t${t}_$i.log 2>&1 || { tail -5 $O/resnet_t${t}_$i.log; exit 1; }
    tail -1 $O/resnet_t${t}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('stem_threads=$t', d['ms_per_step'], d['value'], d['train_loss_mean'])"
  done
done
TAG=r5ap MODEL=resnet50 BATCHES=256 bash tools/gpu/profile.sh
