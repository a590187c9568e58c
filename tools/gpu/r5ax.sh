#!/bin/bash
# round 5: parallel global-avg-pool forward and bias column sums (pool.hip) — kernel tests,
# ResNet tests, ResNet-50 b256 bench x2 + profile
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r5ax; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_resnet.py -k "avgpool or colsum or linear_gemm or resnet50_train_step or bottleneck" -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 10 --ref-window 0 > $O/resnet_$i.log 2>&1 || { tail -5 $O/resnet_$i.log; exit 1; }
  tail -1 $O/resnet_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('resnet', d['ms_per_step'], d['value'])"
done
TAG=r5ax MODEL=resnet50 BATCHES=256 bash tools/gpu/profile.sh
