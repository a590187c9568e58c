#!/bin/bash
# Measurement instruments over the VGG-11 step: the kernel-duration roofline (b256 + b32,
# tools/probes/roofline.py under rocprofv3 --kernel-trace) and the PMC passes (tools/gpu/pmc.sh)
# at b256 and b32, summarised to markdown under gpurun_out/$TAG/.
#   TAG=r6s bash tools/gpu/instruments.sh
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/${TAG:-instr}; mkdir -p $O
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv \
   -d $GRAFT_REPO_ROOT/$O/roof -o r -- python3 $GRAFT_REPO_ROOT/tools/probes/roofline.py --batch 256 32 \
   --trace $GRAFT_REPO_ROOT/$O/roof_phases.json > $GRAFT_REPO_ROOT/$O/roof.log 2>&1) || { tail -5 $O/roof.log; exit 1; }
T=$(find $O/roof -name "r_kernel_trace.csv" | head -1)
python3 tools/probes/roofline_trace.py $O/roof_phases.json $T > $O/roofline_kernels.md || exit 1
rm -rf $O/roof
tail -4 $O/roofline_kernels.md
for B in ${PMC_BATCHES:-256 32}; do
  rm -rf gpurun_out/pmc
  PMC_ARGS="--global-batch $B" timeout -k 10 600 bash tools/gpu/pmc.sh || exit 1
  python3 tools/pmc_summary.py gpurun_out/pmc > $O/pmc_vgg11_b$B.md || exit 1
  rm -rf gpurun_out/pmc
  grep -c "|" $O/pmc_vgg11_b$B.md
done
