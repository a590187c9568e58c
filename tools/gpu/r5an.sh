#!/bin/bash
# round 5: BN-backward reduce over narrower channel chunks (bn_act.hip reduce_split,
# DDP_AMD_BN_REDUCE_GB) — BN kernel tests, ResNet-50 b256 A/B of the chunk width (256 = the
# previous layout), VGG-11 b256 / b32 benches, ResNet kernel profile
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r5an; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -k "bn_act" -x -q --timeout 300 --timeout-method thread > $O/tests_k.log 2>&1 || { tail -30 $O/tests_k.log; exit 1; }
tail -1 $O/tests_k.log
for i in 1 2; do
  for g in 256 32 64; do
    DDP_AMD_BN_REDUCE_GB=$g timeout -k 10 300 python bench.py --model resnet50 --steps 8 --warmup 4 --ref-window 0 > $O/resnet_g${g}_$i.log 2>&1 || { tail -5 $O/resnet_g${g}_$i.log; exit 1; }
    tail -1 $O/resnet_g${g}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('gb=$g', d['ms_per_step'], d['value'], d['train_loss_mean'])"
  done
done
for b in 256 32; do
  for g in 256 32; do
    DDP_AMD_BN_REDUCE_GB=$g timeout -k 10 200 python bench.py --global-batch $b --steps 60 --warmup 10 > $O/b${b}_g$g.log 2>&1 || { tail -5 $O/b${b}_g$g.log; exit 1; }
    tail -1 $O/b${b}_g$g.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('b$b gb=$g', d['ms_per_step'], d['value'])"
  done
done
TAG=r5an MODEL=resnet50 BATCHES=256 bash tools/gpu/profile.sh
