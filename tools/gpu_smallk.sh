#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
timeout -k 10 100 python tools/stats_cost.py || exit 1
bash tools/gpu_quick.sh tests/test_gpu_kernels.py tests/test_gpu_model.py || exit 1
bash tools/gpu_ab.sh X "1" && bash tools/gpu_ab.sh X "1" resnet50
