cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/s || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv_tr.py tests/test_gpu_model.py tests/test_gpu_kernels.py tests/test_gpu_rccl_self.py -x -q --timeout 300 --timeout-method thread > gpurun_out/s/tests.log 2>&1; rc=$?; tail -3 gpurun_out/s/tests.log; [ $rc -eq 0 ] || exit $rc
for P in 1 2; do for B in 32 64; do for T in 32 0; do
  DDP_AMD_FUSE_BN_IN_POOL_MAX_BATCH=$T timeout -k 10 200 python bench.py --global-batch $B --steps 60 --warmup 10 --ref-window 0 > gpurun_out/s/b.log 2>&1 || { tail -5 gpurun_out/s/b.log; exit 1; }
  echo "p$P B=$B POOLMAX=$T $(python -c "import json; d=json.loads(open('gpurun_out/s/b.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['train_loss_mean'])")"
done; done; done
