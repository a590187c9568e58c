#!/bin/bash
# run a subset of GPU tests: bash tools/gpu_quick.sh <pytest args...>
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest "$@" -q -m gpu -p no:cacheprovider -rA > gpurun_out/pytest_quick.log 2>&1
rc=$?; grep -E "passed|failed|error|^E  |cos|\{" gpurun_out/pytest_quick.log | tail -30; echo "pytest rc=$rc"
exit $rc
