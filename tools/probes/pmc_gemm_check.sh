#!/bin/bash
# PMC normalisation check on the standalone GEMM structure probe (no torch): SQ_VALU_MFMA_BUSY_CYCLES
# and SQ_INSTS_MFMA per dispatch vs the dispatch's own FLOPs and kernel duration
# (tools/pmc_summary.py --gemm-check). One --pmc pass (<= 8 SQ, 2 GRBM counters).
cd "$GRAFT_REPO_ROOT" || exit 2
O=$GRAFT_REPO_ROOT/gpurun_out/pmcgemm; mkdir -p $O
hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probes/gemm_struct.hip -o /tmp/gemm_struct || exit 1
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --kernel-trace \
   --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
   --output-format csv -d $O/p1 -o g -- /tmp/gemm_struct 5 > $O/struct.jsonl 2> $O/struct.err) || { tail -5 $O/struct.err; exit 1; }
tail -3 $O/struct.jsonl
