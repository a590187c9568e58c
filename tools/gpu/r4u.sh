#!/bin/bash
# round 4: L0 weight gradient fused into the dz pass — kernel tests, model tests, A/B, profiles
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r4u; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "l0_fused or sgd_in_backward" -x -v --timeout 120 --timeout-method thread > $O/k1.log 2>&1 || { grep -E "FAIL|Error|assert" $O/k1.log | head -20; tail -30 $O/k1.log; exit 1; }
tail -1 $O/k1.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py -x -q --timeout 300 --timeout-method thread > $O/k2.log 2>&1 || { grep -E "FAIL|Error" $O/k2.log | head -20; tail -30 $O/k2.log; exit 1; }
tail -1 $O/k2.log
for P in 1 2; do
for CFG in 256 32; do
  for V in "base:" "nowg:DDP_AMD_L0_WGRAD=0"; do
    NAME=${V%%:*}; ENVS=${V#*:}
    L=$O/b${CFG}_${NAME}_p$P.log
    env $ENVS timeout -k 10 200 python bench.py --global-batch $CFG --steps 60 --warmup 10 --ref-window 0 > $L 2>&1 || { tail -5 $L; exit 1; }
    echo "b$CFG $NAME p$P $(python -c "import json; d=json.loads(open('$L').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['train_loss_mean'])")"
  done
done
done
TAG=r4u BATCHES="256 32" bash tools/gpu/profile.sh || exit 1
for f in r4u_vgg11_b256 r4u_vgg11_b32; do echo $f; grep "l0_" gpurun_out/prof/$f.md | grep "^| [0-9]" ; done
