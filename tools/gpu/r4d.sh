#!/bin/bash
# round 4: kernel tests of the new paths (XF conv backward, SGD in the backward, k-major
# tap-reuse dgrad), the model tests, a same-session A/B of the defaults, step profiles
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r4d; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_conv_tr.py -k "xf or sgd_in_backward or tr_wc" -x -v --timeout 120 --timeout-method thread > $O/k1.log 2>&1 || { grep -E "FAIL|Error" $O/k1.log | head -20; tail -30 $O/k1.log; exit 1; }
tail -1 $O/k1.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_model.py -x -v --timeout 300 --timeout-method thread > $O/k2.log 2>&1 || { grep -E "FAIL|Error" $O/k2.log | head -20; tail -30 $O/k2.log; exit 1; }
tail -1 $O/k2.log
grep -A14 "lr01_headline" $O/k2.log | grep -E "^(fused|emu|fp32|k0|step)" | head -14
for CFG in 256 32; do
  for V in "base:" "noxf:DDP_AMD_BN_BWD_XF=0" "nosgd:DDP_AMD_SGD_IN_BWD=0" "trdg:DDP_AMD_DGRAD_TR=1"; do
    NAME=${V%%:*}; ENVS=${V#*:}
    L=$O/b${CFG}_$NAME.log
    env $ENVS timeout -k 10 200 python bench.py --global-batch $CFG --steps 60 --warmup 10 --ref-window 0 > $L 2>&1 || { tail -5 $L; exit 1; }
    echo "b$CFG $NAME $(python -c "import json; d=json.loads(open('$L').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['train_loss_mean'])")"
  done
done
TAG=r4d BATCHES="256 32" bash tools/gpu/profile.sh || exit 1
