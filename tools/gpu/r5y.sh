#!/bin/bash
# round 5: SGD on the fp32 master inside the backward pairs' unsplit WGRAD epilogue (one GPU,
# conv_igemm.hip ConvArgs::sgd; operand re-pack = optim.hip item 5) — SGD / model /
# deterministic tests, VGG-11 b32 and b256 A/B (DDP_AMD_SGD_PAIR_MASTER=0 vs 1)
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r5y; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_deterministic.py tests/test_gpu_kernels.py -k "sgd or deterministic or trajectory or graph or oracle" -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAIL|Error" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for b in 32 256; do
  for i in 1 2 3; do
    for m in 0 1; do
      DDP_AMD_SGD_PAIR_MASTER=$m timeout -k 10 200 python bench.py --global-batch $b --steps 60 --warmup 10 > $O/vgg_b${b}_m${m}_$i.log 2>&1 || { tail -5 $O/vgg_b${b}_m${m}_$i.log; exit 1; }
      tail -1 $O/vgg_b${b}_m${m}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('b$b master=$m', d['ms_per_step'], d['value'], d['train_loss_mean'])"
    done
  done
done
