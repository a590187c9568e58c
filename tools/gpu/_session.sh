cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/s || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "bn_act" -x -q --timeout 200 --timeout-method thread > gpurun_out/s/tests.log 2>&1; rc=$?; tail -3 gpurun_out/s/tests.log; [ $rc -eq 0 ] || { grep -m8 "Error\|assert\|FAIL" gpurun_out/s/tests.log; exit $rc; }
NOTEST=1 VARIANTS="off:DDP_AMD_BN_BWD_CLUSTER=0 on:DDP_AMD_BN_BWD_CLUSTER=1" CFGS="vgg11:32 vgg11:64 vgg11:128 vgg11:256" bash tools/gpu/ab_env.sh && TAG=r3d BATCHES="32" bash tools/gpu/profile.sh
