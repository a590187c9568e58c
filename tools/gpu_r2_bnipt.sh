#!/bin/bash
# BN-backward grid sizing on ResNet-50 b256: target blocks x max items per thread
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/bnipt
for P in 1 2; do
  for CFG in 1024:4 1024:16 512:16 256:16 2048:8; do
    BL=${CFG%%:*}; IP=${CFG##*:}
    L=gpurun_out/bnipt/rn_${BL}_${IP}_p$P.log
    DDP_AMD_BN_BWD_BLOCKS=$BL DDP_AMD_BN_BWD_MAX_IPT=$IP timeout -k 10 200 python bench.py --model resnet50 --steps 20 --warmup 8 --ref-window 0 > $L 2>&1 || { tail -5 $L; exit 1; }
    echo "blocks=$BL ipt<=$IP p$P $(python -c "import json; d=json.loads(open('$L').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['train_loss_mean'])")"
  done
done
