#!/bin/bash
# round 4: dense 2x2 pair keeps the measured WGRAD split (its finish takes the SGD step): tests, A/B, profile
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r4o; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "dense2x2 or sgd_in_backward or l0_fused or bwd_pair" -x -q --timeout 120 --timeout-method thread > $O/k1.log 2>&1 || { grep -E "FAIL|Error|assert" $O/k1.log | head -20; tail -30 $O/k1.log; exit 1; }
tail -1 $O/k1.log
for P in 1 2; do
for CFG in 256 128 32; do
  for V in "base:" "nod2:DDP_AMD_DENSE2X2=0"; do
    NAME=${V%%:*}; ENVS=${V#*:}
    L=$O/b${CFG}_${NAME}_p$P.log
    env $ENVS timeout -k 10 200 python bench.py --global-batch $CFG --steps 60 --warmup 10 --ref-window 0 > $L 2>&1 || { tail -5 $L; exit 1; }
    echo "b$CFG $NAME p$P $(python -c "import json; d=json.loads(open('$L').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['train_loss_mean'])")"
  done
done
done
TAG=r4o BATCHES="256 32" bash tools/gpu/profile.sh || exit 1
