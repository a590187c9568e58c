#!/bin/bash
# round 5: deferred residual gradient for ResNet identity blocks (GradLink.defer, conv_igemm.hip
# ConvArgs::acc_dy / acc_mask) — kernel numerics, ResNet tests, ResNet-50 b256 A/B
# (DDP_AMD_RES_DEFER=0 vs 1, interleaved)
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r5l; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -k "deferred_branch or bn_act_fwd_bwd or staged_epilogue" -x -q --timeout 300 --timeout-method thread > $O/tests_k.log 2>&1 || { grep -E "FAIL|Error" $O/tests_k.log | head; tail -30 $O/tests_k.log; exit 1; }
tail -1 $O/tests_k.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_resnet.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAIL|Error" $O/tests.log | head -20; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for m in 0 1; do
    DDP_AMD_RES_DEFER=$m timeout -k 10 300 python bench.py --model resnet50 --steps 8 --warmup 4 --ref-window 0 > $O/resnet_d${m}_$i.log 2>&1 || { tail -5 $O/resnet_d${m}_$i.log; exit 1; }
    tail -1 $O/resnet_d${m}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('defer=$m', d['ms_per_step'], d['value'], d['train_loss_mean'])"
  done
done
