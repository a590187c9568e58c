#!/bin/bash
# round 5: VGG-11 with the re-tuned conv table (tools/gpu/conv_tuning_r5s.json, r5s) vs the
# shipped one, b256 and b32, interleaved
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r5t; mkdir -p $O
NEW=$GRAFT_REPO_ROOT/tools/gpu/conv_tuning_r5s.json
for b in 256 32; do
  for i in 1 2 3; do
    for m in old new; do
      if [ $m = new ]; then export DDP_AMD_CONV_TUNING_FILE=$NEW; else unset DDP_AMD_CONV_TUNING_FILE; fi
      timeout -k 10 200 python bench.py --global-batch $b --steps 60 --warmup 10 > $O/vgg_b${b}_${m}_$i.log 2>&1 || { tail -5 $O/vgg_b${b}_${m}_$i.log; exit 1; }
      tail -1 $O/vgg_b${b}_${m}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('b$b table=$m', d['ms_per_step'], d['value'])"
    done
  done
done
