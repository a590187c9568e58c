#!/bin/bash
# PMC counters for the per-layer conv micro-benchmark (separate passes; --pmc only with
# --kernel-trace). Usage: gpurun -- bash tools/gpu_pmc_conv.sh [vgg11|resnet50]
cd "$GRAFT_REPO_ROOT" || exit 2
root="$GRAFT_REPO_ROOT"
model="${1:-vgg11}"
mkdir -p gpurun_out/pmc_conv
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVES" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  i=$((i+1))
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set \
      --output-format csv -d "$root/gpurun_out/pmc_conv/p$i" -o conv -- \
      python3 "$root/tools/conv_bench.py" --model "$model" --reps 2 > "$root/gpurun_out/pmc_conv/p$i.log" 2>&1)
  rc=$?; echo "pass $i rc=$rc"; tail -1 gpurun_out/pmc_conv/p$i.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
exit 0
