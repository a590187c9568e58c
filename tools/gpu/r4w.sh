#!/bin/bash
# round 4: last block's BN + ReLU + pool folded into the head's forward — model tests, A/B, profile
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r4w; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_kernels.py -k "not every_tile" -x -q --timeout 300 --timeout-method thread > $O/k.log 2>&1 || { grep -E "FAIL|Error" $O/k.log | head -20; tail -30 $O/k.log; exit 1; }
tail -1 $O/k.log
for P in 1 2; do
for CFG in 256 128 32; do
  for V in "base:" "nohb:DDP_AMD_HEAD_BN_FWD=0"; do
    NAME=${V%%:*}; ENVS=${V#*:}
    L=$O/b${CFG}_${NAME}_p$P.log
    env $ENVS timeout -k 10 200 python bench.py --global-batch $CFG --steps 60 --warmup 10 --ref-window 0 > $L 2>&1 || { tail -5 $L; exit 1; }
    echo "b$CFG $NAME p$P $(python -c "import json; d=json.loads(open('$L').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['train_loss_mean'])")"
  done
done
done
TAG=r4w BATCHES="256" bash tools/gpu/profile.sh || exit 1
