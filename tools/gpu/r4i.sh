#!/bin/bash
# round 4: L0 block v3 — operand prefetch A/B (DDP_AMD_L0_PF), kernel test, profiles
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r4i; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "l0_fused" -x -v --timeout 120 --timeout-method thread > $O/k1.log 2>&1 || { grep -E "FAIL|Error|assert" $O/k1.log | head -20; tail -30 $O/k1.log; exit 1; }
tail -1 $O/k1.log
DDP_AMD_L0_PF=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "l0_fused" -x -q --timeout 120 --timeout-method thread > $O/k1b.log 2>&1 || { tail -30 $O/k1b.log; exit 1; }
tail -1 $O/k1b.log
for P in 1 2; do
for CFG in 256 32; do
  for V in "base:" "pf0:DDP_AMD_L0_PF=0" "nol0:DDP_AMD_L0_FUSE=0"; do
    NAME=${V%%:*}; ENVS=${V#*:}
    L=$O/b${CFG}_${NAME}_p$P.log
    env $ENVS timeout -k 10 200 python bench.py --global-batch $CFG --steps 60 --warmup 10 --ref-window 0 > $L 2>&1 || { tail -5 $L; exit 1; }
    echo "b$CFG $NAME p$P $(python -c "import json; d=json.loads(open('$L').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['train_loss_mean'])")"
  done
done
done
TAG=r4i BATCHES="256 32" bash tools/gpu/profile.sh || exit 1
TAG=r4i_pf0 ENVS="DDP_AMD_L0_PF=0" BATCHES="256 32" bash tools/gpu/profile.sh || exit 1
for f in r4i_vgg11_b256 r4i_pf0_vgg11_b256 r4i_vgg11_b32 r4i_pf0_vgg11_b32; do echo $f; grep "l0_" gpurun_out/prof/$f.md | grep -v "^| [0-9]" ; done
