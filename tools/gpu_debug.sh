#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
timeout -k 10 300 python tools/debug_vgg.py > gpurun_out/debug_vgg.log 2>&1
rc=$?; cat gpurun_out/debug_vgg.log | grep -v amdgpu.ids; echo "debug rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_check.sh tests bench
