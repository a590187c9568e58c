#!/bin/bash
# round 5: ordering check of the tree A/B (r5ah): current tree FIRST in each pair, then the
# session-start tree (_oldtree/), VGG-11 b256
cd "$GRAFT_REPO_ROOT" || exit 2
O=$GRAFT_REPO_ROOT/gpurun_out/r5ai; mkdir -p $O
for i in 1 2 3 4; do
  for t in new old; do
    if [ $t = old ]; then D=$GRAFT_REPO_ROOT/_oldtree; else D=$GRAFT_REPO_ROOT; fi
    (cd $D && timeout -k 10 200 python bench.py --steps 60 --warmup 10 > $O/b256_${t}_$i.log 2>&1) || { tail -5 $O/b256_${t}_$i.log; exit 1; }
    tail -1 $O/b256_${t}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('b256 $t', d['ms_per_step'], d['value'])"
  done
done
