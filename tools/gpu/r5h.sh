#!/bin/bash
# round 5: measurement instruments — PMC normalisation check on the GEMM structure probe, the
# kernel-duration roofline (b256 + b32), PMC passes over the VGG-11 b256 step
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r5h; mkdir -p $O
bash tools/probes/pmc_gemm_check.sh || exit 1
python3 tools/pmc_summary.py --gemm-check gpurun_out/pmcgemm gpurun_out/pmcgemm/struct.jsonl 5 > $O/pmc_gemm_check.md || exit 1
head -8 $O/pmc_gemm_check.md
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv \
   -d $GRAFT_REPO_ROOT/$O/roof -o r -- python3 $GRAFT_REPO_ROOT/tools/probes/roofline.py --batch 256 32 \
   --trace $GRAFT_REPO_ROOT/$O/roof_phases.json > $GRAFT_REPO_ROOT/$O/roof.log 2>&1) || { tail -5 $O/roof.log; exit 1; }
T=$(find $O/roof -name "r_kernel_trace.csv" | head -1)
python3 tools/probes/roofline_trace.py $O/roof_phases.json $T > $O/roofline_kernels.md || exit 1
tail -4 $O/roofline_kernels.md
rm -rf gpurun_out/pmc
timeout -k 10 600 bash tools/gpu/pmc.sh || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc > $O/pmc_vgg11_b256.md || exit 1
grep -c "|" $O/pmc_vgg11_b256.md
