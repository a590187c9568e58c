#!/bin/bash
# round 5: the 2x2 no-pool block's BN backward inside the next dgrad's split-K finish at <= 128
# rows (ops/layers.py bn_bwd_fuse_pays; DDP_AMD_BN_BWD_NOPOOL_SMALL=0 = separate pass) —
# model tests, VGG-11 b32 / b64 A/B
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r5z; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_model.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAIL|Error" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for b in 32 64; do
  for i in 1 2 3; do
    for m in 0 1; do
      DDP_AMD_BN_BWD_NOPOOL_SMALL=$m timeout -k 10 200 python bench.py --global-batch $b --steps 60 --warmup 10 > $O/vgg_b${b}_m${m}_$i.log 2>&1 || { tail -5 $O/vgg_b${b}_m${m}_$i.log; exit 1; }
      tail -1 $O/vgg_b${b}_m${m}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('b$b nopool=$m', d['ms_per_step'], d['value'], d['train_loss_mean'])"
    done
  done
done
