#!/bin/bash
# round 5: BN-backward fold threshold 32 vs 64 MB (DDP_AMD_BN_FOLD_BWD_MB), VGG-11 b256 / b128
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r5aa; mkdir -p $O
for b in 256 128; do
  for i in 1 2 3; do
    for m in 32 64; do
      DDP_AMD_BN_FOLD_BWD_MB=$m timeout -k 10 200 python bench.py --global-batch $b --steps 60 --warmup 10 > $O/vgg_b${b}_f${m}_$i.log 2>&1 || { tail -5 $O/vgg_b${b}_f${m}_$i.log; exit 1; }
      tail -1 $O/vgg_b${b}_f${m}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('b$b fold=$m', d['ms_per_step'], d['value'])"
    done
  done
done
