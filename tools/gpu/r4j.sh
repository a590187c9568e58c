#!/bin/bash
# round 4: L0 block v4 — DPP-bitmask pool argmax, folded BN-backward coefficients; grid cap A/B
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r4j; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "l0_fused" -x -v --timeout 120 --timeout-method thread > $O/k1.log 2>&1 || { grep -E "FAIL|Error|assert" $O/k1.log | head -20; tail -30 $O/k1.log; exit 1; }
tail -1 $O/k1.log
for P in 1 2; do
for CFG in 256 32; do
  for V in "base:" "g2048:DDP_AMD_L0_BLOCKS=2048" "g512:DDP_AMD_L0_BLOCKS=512" "nol0:DDP_AMD_L0_FUSE=0"; do
    NAME=${V%%:*}; ENVS=${V#*:}
    L=$O/b${CFG}_${NAME}_p$P.log
    env $ENVS timeout -k 10 200 python bench.py --global-batch $CFG --steps 60 --warmup 10 --ref-window 0 > $L 2>&1 || { tail -5 $L; exit 1; }
    echo "b$CFG $NAME p$P $(python -c "import json; d=json.loads(open('$L').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['train_loss_mean'])")"
  done
done
done
TAG=r4j BATCHES="256 32" bash tools/gpu/profile.sh || exit 1
TAG=r4j_g4096 ENVS="DDP_AMD_L0_BLOCKS=4096" BATCHES="256" bash tools/gpu/profile.sh || exit 1
for f in r4j_vgg11_b256 r4j_g4096_vgg11_b256 r4j_vgg11_b32; do echo $f; grep "l0_" gpurun_out/prof/$f.md | grep -v "^| [0-9]" ; done
