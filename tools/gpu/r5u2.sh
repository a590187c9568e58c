#!/bin/bash
# round 5: VGG-11 b256 A/B of DDP_AMD_FWD_STAT_GRID (r5u follow-up, 4 interleaved pairs)
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r5u2; mkdir -p $O
for i in 1 2 3 4; do
  for m in 0 2048; do
    DDP_AMD_FWD_STAT_GRID=$m timeout -k 10 200 python bench.py --steps 60 --warmup 10 > $O/vgg_g${m}_$i.log 2>&1 || { tail -5 $O/vgg_g${m}_$i.log; exit 1; }
    tail -1 $O/vgg_g${m}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('vgg grid=$m', d['ms_per_step'], d['value'])"
  done
done
