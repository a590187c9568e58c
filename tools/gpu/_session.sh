cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/tr || exit 1
timeout -k 10 900 python -u tools/conv_tune_tr.py --batch 256 128 64 32 --write --out gpurun_out/tr/conv_tuning.json > gpurun_out/tr/sweep_all.jsonl 2> gpurun_out/tr/sweep_all.err || { tail -5 gpurun_out/tr/sweep_all.err; exit 1; }
tail -1 gpurun_out/tr/sweep_all.jsonl
for B in 256 32 64 128; do for T in 1 0; do
  DDP_AMD_CONV_TUNING_FILE=gpurun_out/tr/conv_tuning.json DDP_AMD_CONV_TR=$T timeout -k 10 200 python bench.py --global-batch $B --steps 60 --warmup 10 --ref-window 0 > gpurun_out/tr/bench_${B}_$T.log 2>&1 || { tail -5 gpurun_out/tr/bench_${B}_$T.log; exit 1; }
  echo "B=$B TR=$T $(python -c "import json; d=json.loads(open('gpurun_out/tr/bench_${B}_$T.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['train_loss_mean'])")"
done; done
