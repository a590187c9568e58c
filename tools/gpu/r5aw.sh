#!/bin/bash
# round 5: strided shortcut dgrad deferred behind the other branch (GradLink.deferred_dgrad,
# DDP_AMD_DS_DGRAD_DEFER) — ResNet tests, accumulate-dgrad kernel tests, ResNet-50 b256 A/B
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r5aw; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_resnet.py tests/test_gpu_kernels.py -k "resnet or bottleneck or staged_epilogue or dgrad" -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAIL|Error" $O/tests.log | head -20; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for d in 0 1; do
    DDP_AMD_DS_DGRAD_DEFER=$d timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 10 --ref-window 0 > $O/resnet_d${d}_$i.log 2>&1 || { tail -5 $O/resnet_d${d}_$i.log; exit 1; }
    tail -1 $O/resnet_d${d}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('defer=$d', d['ms_per_step'], d['value'], d['train_loss_mean'])"
  done
done
TAG=r5aw MODEL=resnet50 BATCHES=256 bash tools/gpu/profile.sh
