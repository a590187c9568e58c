#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -q -m gpu -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after pytest rc=$rc"; exit $rc; fi
timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/bench1.log 2>&1
rc=$?
echo "bench rc=$rc"; tail -20 gpurun_out/bench1.log
exit $rc
