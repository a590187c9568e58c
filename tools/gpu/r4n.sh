#!/bin/bash
# round 4: dense 2x2 conv form — kernel test, conv + model tests, A/B (DDP_AMD_DENSE2X2=0), profiles
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r4n; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "dense2x2" -x -v --timeout 120 --timeout-method thread > $O/k1.log 2>&1 || { grep -E "FAIL|Error|assert" $O/k1.log | head -20; tail -30 $O/k1.log; exit 1; }
tail -1 $O/k1.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { grep -E "FAIL|Error" $O/gpu_tests.log | head -20; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
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
TAG=r4n BATCHES="256 32" bash tools/gpu/profile.sh || exit 1
