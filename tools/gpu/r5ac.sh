#!/bin/bash
# round 5: b32 forward 4x4 tap-reuse convs unsplit (no split-K finish launch) vs the tuned split 4
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r5ac; mkdir -p $O
# (NEW: the shipped table with the two N32 4x4 tr_entries set to splits 1, written to this path for the run)
NEW=$GRAFT_REPO_ROOT/tools/gpu/conv_tuning_tr_nosplit.json
for i in 1 2 3; do
  for m in old new; do
    if [ $m = new ]; then export DDP_AMD_CONV_TUNING_FILE=$NEW; else unset DDP_AMD_CONV_TUNING_FILE; fi
    timeout -k 10 200 python bench.py --global-batch 32 --steps 60 --warmup 10 > $O/b32_${m}_$i.log 2>&1 || { tail -5 $O/b32_${m}_$i.log; exit 1; }
    tail -1 $O/b32_${m}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('b32 table=$m', d['ms_per_step'], d['value'])"
  done
done
