#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_resnet.py tests/test_gpu_kernels.py -q -m gpu -p no:cacheprovider -rA > gpurun_out/pytest_resnet.log 2>&1
rc=$?; grep -E "passed|failed|error|^E  " gpurun_out/pytest_resnet.log | tail -15; echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_vgg.log 2>&1
rc=$?; tail -1 gpurun_out/bench_vgg.log; echo "bench vgg rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --model resnet50 --steps 10 --warmup 3 > gpurun_out/bench_resnet.log 2>&1
rc=$?; tail -3 gpurun_out/bench_resnet.log; echo "bench resnet rc=$rc"
exit $rc
