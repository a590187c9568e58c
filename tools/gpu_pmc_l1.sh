#!/bin/bash
# L1 (TCP) vs L2 (TCC) traffic of the VGG conv kernels: how much of the implicit-GEMM tap re-reads
# does the vector L1 absorb? Usage: gpurun -- bash tools/gpu_pmc_l1.sh
cd "$GRAFT_REPO_ROOT" || exit 2
root="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc_l1
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 60 rocprofv3 -L > "$root/gpurun_out/pmc_l1/counters.txt" 2>&1)
grep -o -E "(TCP|TCC|TA|TD)_[A-Z0-9_]*" gpurun_out/pmc_l1/counters.txt | sort -u > gpurun_out/pmc_l1/names.txt
wc -l gpurun_out/pmc_l1/names.txt
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_REQ_sum TCC_HIT_sum \
    --output-format csv -d "$root/gpurun_out/pmc_l1/p1" -o conv -- \
    python3 "$root/tools/conv_bench.py" --model vgg11 --reps 2 > "$root/gpurun_out/pmc_l1/p1.log" 2>&1)
rc=$?; echo "pass rc=$rc"; tail -2 gpurun_out/pmc_l1/p1.log
exit $rc
