#!/bin/bash
# round-4 start: live-RCCL tests (captured 2A/2B, stage profiling), every-tile conv test, then
# step profiles at 256/128/64/32
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/r4a
timeout -k 10 400 python -u -m pytest tests/test_gpu_rccl_self.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r4a/rccl_tests.log 2>&1 || { tail -40 gpurun_out/r4a/rccl_tests.log; exit 1; }
tail -2 gpurun_out/r4a/rccl_tests.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -k every_tile -v --timeout 200 --timeout-method thread > gpurun_out/r4a/tile_tests.log 2>&1; echo "tile tests rc=$?"; grep -E "PASS|FAIL" gpurun_out/r4a/tile_tests.log | tail -40
TAG=r4start BATCHES="256 128 64 32" bash tools/gpu/profile.sh
