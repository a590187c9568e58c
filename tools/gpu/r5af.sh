#!/bin/bash
# round 5: this session's tree vs the session-start tree (commit 3728385, built in _oldtree/),
# same box, interleaved: VGG-11 b256 / b32 and ResNet-50 b256
cd "$GRAFT_REPO_ROOT" || exit 2
O=$GRAFT_REPO_ROOT/gpurun_out/r5af; mkdir -p $O
for i in 1 2 3; do
  for t in old new; do
    if [ $t = old ]; then D=$GRAFT_REPO_ROOT/_oldtree; else D=$GRAFT_REPO_ROOT; fi
    (cd $D && timeout -k 10 200 python bench.py --steps 60 --warmup 10 > $O/b256_${t}_$i.log 2>&1) || { tail -5 $O/b256_${t}_$i.log; exit 1; }
    tail -1 $O/b256_${t}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('b256 $t', d['ms_per_step'], d['value'])"
    (cd $D && timeout -k 10 200 python bench.py --global-batch 32 --steps 60 --warmup 10 > $O/b32_${t}_$i.log 2>&1) || { tail -5 $O/b32_${t}_$i.log; exit 1; }
    tail -1 $O/b32_${t}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('b32 $t', d['ms_per_step'], d['value'])"
  done
done
for t in old new; do
  if [ $t = old ]; then D=$GRAFT_REPO_ROOT/_oldtree; else D=$GRAFT_REPO_ROOT; fi
  (cd $D && timeout -k 10 300 python bench.py --model resnet50 --steps 8 --warmup 4 --ref-window 0 > $O/resnet_${t}.log 2>&1) || { tail -5 $O/resnet_${t}.log; exit 1; }
  tail -1 $O/resnet_${t}.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('resnet $t', d['ms_per_step'], d['value'])"
done
