#!/bin/bash
# Re-tune the VGG-11 FWD/DGRAD/WGRAD tile / split-K table on the current kernels (batched
# finishes), merged into the shipped table (pair and ResNet entries kept), then bench A/B
# shipped vs re-tuned at b32/b64/b128/b256, two passes.
cd "$GRAFT_REPO_ROOT" || exit 2
OUT=gpurun_out/vt
mkdir -p $OUT
T=distributed-data-parallel-ml-training_amd/ops/conv_tuning.json
timeout -k 10 700 python -u tools/conv_tune.py --sets vgg --reps 20 --merge $T --out $OUT/conv_tuning_vgg.json > $OUT/tune.log 2>&1 || { tail -20 $OUT/tune.log; exit 1; }
tail -1 $OUT/tune.log
for P in 1 2; do
for B in 32 64 128 256; do
  for V in base vgg; do
    F=$T; [ $V = vgg ] && F=$OUT/conv_tuning_vgg.json
    L=$OUT/b${B}_${V}_p$P.log
    DDP_AMD_CONV_TUNING_FILE=$F timeout -k 10 120 python bench.py --global-batch $B --steps 60 --warmup 10 --ref-window 0 > $L 2>&1 || { tail -5 $L; exit 1; }
    echo "B=$B $V p$P $(python -c "import json; d=json.loads(open('$L').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['train_loss_mean'])")"
  done
done
done
