#!/bin/bash
# PMC counters for the VGG-11 step (separate passes; --pmc only with --kernel-trace/--stats;
# per pass at most 8 SQ, 4 TCC (FETCH_SIZE takes 3), 2 GRBM counters).
cd "$GRAFT_REPO_ROOT" || exit 2
root="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES" \
           "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" \
           "FETCH_SIZE GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set \
      --output-format csv -d "$root/gpurun_out/pmc/p$i" -o vgg -- \
      python3 "$root/bench.py" --steps 3 --warmup 2 --ref-window 0 ${PMC_ARGS:-} > "$root/gpurun_out/pmc/p$i.log" 2>&1)
  rc=$?; echo "pass $i rc=$rc"; tail -1 gpurun_out/pmc/p$i.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
