#!/bin/bash
# round 5: backward-pair re-tune at 32 / 64 images on the round-5 kernels, then in-step A/B
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r5ad; mkdir -p $O
timeout -k 10 900 python -u tools/conv_tune.py --pairs --pair-sets "vgg11:32,64" --reps 30 --merge distributed-data-parallel-ml-training_amd/ops/conv_tuning.json --out $O/conv_tuning.json > $O/tune.log 2>&1 || { tail -20 $O/tune.log; exit 1; }
cat $O/tune.log | tail -20
for b in 32 64; do
  for i in 1 2 3; do
    for m in old new; do
      if [ $m = new ]; then export DDP_AMD_CONV_TUNING_FILE=$GRAFT_REPO_ROOT/$O/conv_tuning.json; else unset DDP_AMD_CONV_TUNING_FILE; fi
      timeout -k 10 200 python bench.py --global-batch $b --steps 60 --warmup 10 > $O/b${b}_${m}_$i.log 2>&1 || { tail -5 $O/b${b}_${m}_$i.log; exit 1; }
      tail -1 $O/b${b}_${m}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('b$b table=$m', d['ms_per_step'], d['value'])"
    done
  done
done
