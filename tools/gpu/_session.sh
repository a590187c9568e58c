cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/tr || exit 1
for P in 1 2; do
for B in 256 128 64 32; do for T in 1 0; do
  DDP_AMD_DGRAD_TR=$T timeout -k 10 200 python bench.py --global-batch $B --steps 60 --warmup 10 --ref-window 0 > gpurun_out/tr/b.log 2>&1 || { tail -5 gpurun_out/tr/b.log; exit 1; }
  echo "p$P B=$B DGRAD_TR=$T $(python -c "import json; d=json.loads(open('gpurun_out/tr/b.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['train_loss_mean'])")"
done; done; done
timeout -k 10 900 python -u -m pytest tests/test_gpu_conv_tr.py tests/test_gpu_model.py tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tr/tests.log 2>&1; rc=$?; tail -3 gpurun_out/tr/tests.log; [ $rc -eq 0 ] || exit $rc
