#!/bin/bash
# round 5: ResNet-50 b256 with the r5o / r5q table (stem WGRAD split-K 512, accumulate DGRAD 128x64, ResNet re-tune
# 128x64) vs the table before them, interleaved
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/${TAG:-r5p}; mkdir -p $O
# (OLD: the table of the commit before, copied to tools/gpu/conv_tuning_before_r5o.json for the run)
OLD=$GRAFT_REPO_ROOT/tools/gpu/conv_tuning_before_r5o.json
for i in 1 2; do
  for m in old new; do
    if [ $m = old ]; then export DDP_AMD_CONV_TUNING_FILE=$OLD; else unset DDP_AMD_CONV_TUNING_FILE; fi
    timeout -k 10 300 python bench.py --model resnet50 --steps 8 --warmup 4 --ref-window 0 > $O/resnet_${m}_$i.log 2>&1 || { tail -5 $O/resnet_${m}_$i.log; exit 1; }
    tail -1 $O/resnet_${m}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('table=$m', d['ms_per_step'], d['value'], d['train_loss_mean'])"
  done
done
unset DDP_AMD_CONV_TUNING_FILE
timeout -k 10 600 python -u -m pytest tests/test_gpu_resnet.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
