#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r4z13; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_bench_contract.py -v --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
grep -E "PASS|FAIL" $O/t.log
