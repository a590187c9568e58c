#!/bin/bash
# round 5: the input block's BN-backward sums in conv1's dgrad finish (DDP_AMD_L0_SUMS_IN_FINISH)
# + BN-backward fold threshold 32 / 64 MB (DDP_AMD_BN_FOLD_BWD_MB) — tests, VGG-11 A/B
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r5ab; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_kernels.py tests/test_gpu_deterministic.py -k "l0 or oracle or trajectory or graph or sgd or deterministic or bn_act" -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAIL|Error" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for b in 32 256; do
  for i in 1 2 3; do
    for m in 0 1; do
      DDP_AMD_L0_SUMS_IN_FINISH=$m timeout -k 10 200 python bench.py --global-batch $b --steps 60 --warmup 10 > $O/vgg_b${b}_l${m}_$i.log 2>&1 || { tail -5 $O/vgg_b${b}_l${m}_$i.log; exit 1; }
      tail -1 $O/vgg_b${b}_l${m}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('b$b l0fin=$m', d['ms_per_step'], d['value'], d['train_loss_mean'])"
    done
  done
done
for b in 256 128; do
  for i in 1 2; do
    for m in 32 64; do
      DDP_AMD_BN_FOLD_BWD_MB=$m timeout -k 10 200 python bench.py --global-batch $b --steps 60 --warmup 10 > $O/vgg_b${b}_f${m}_$i.log 2>&1 || { tail -5 $O/vgg_b${b}_f${m}_$i.log; exit 1; }
      tail -1 $O/vgg_b${b}_f${m}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('b$b fold=$m', d['ms_per_step'], d['value'])"
    done
  done
done
