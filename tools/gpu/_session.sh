cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/trpmc && root=$GRAFT_REPO_ROOT
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES"; do
  i=$((i+1))
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $set --output-format csv -d "$root/gpurun_out/trpmc/p$i" -o t -- python3 "$root/tools/probes/tr_probe.py" 32 512 512 2 64 64 1 3 > "$root/gpurun_out/trpmc/p$i.log" 2>&1) || { tail -5 gpurun_out/trpmc/p$i.log; exit 1; }
done
python3 tools/pmc_summary.py gpurun_out/trpmc
