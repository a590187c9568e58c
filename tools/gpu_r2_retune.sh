#!/bin/bash
# re-run the conv tile/stage/split sweep on the round-2 kernels (VGG-11 at 256/128/64/32)
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/tune
timeout -k 10 1100 python -u tools/conv_tune.py --sets all --reps 20 --out gpurun_out/tune/conv_tuning_r2.json > gpurun_out/tune/tune.log 2>&1 || { tail -5 gpurun_out/tune/tune.log; exit 1; }
tail -2 gpurun_out/tune/tune.log
