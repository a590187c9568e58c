#!/bin/bash
# PMC passes over the ResNet-50 layer1 conv3 forward (1x1, 64 -> 256 channels, 56x56, N=256)
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc64
i=0
SETS=${PMC_SETS:-all}
if [ "$SETS" = insts ]; then
  LIST=("SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS")
else
  LIST=("SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY"
        "WRITE_SIZE GRBM_GUI_ACTIVE" "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum")
fi
for C in "${LIST[@]}"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmc64/${SETS}_p$i -o run -- python3 tools/stat_probe.py --only "64-> 256" --nostats --reps 5 > gpurun_out/pmc64/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc64/p$i.log; exit 1; }
done
echo ok
