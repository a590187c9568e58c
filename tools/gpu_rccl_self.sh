#!/bin/bash
# Live single-rank RCCL communicators on one GPU: the collective paths of the multi-GPU step
# (RCCL inside captured graphs, segmented step's second communicator) + their bench cost.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_rccl_self.py -x -v --timeout 120 --timeout-method thread > gpurun_out/rccl_self_tests.log 2>&1 || { tail -40 gpurun_out/rccl_self_tests.log; exit 1; }
tail -3 gpurun_out/rccl_self_tests.log
for seg in 0 4; do
  DDP_AMD_RCCL_SELF=1 timeout -k 10 200 python bench.py --segmented $seg > gpurun_out/bench_self_seg$seg.log 2>&1 || { tail -20 gpurun_out/bench_self_seg$seg.log; exit 1; }
  tail -1 gpurun_out/bench_self_seg$seg.log
done
for st in allreduce gather_scatter; do
  DDP_AMD_RCCL_SELF=1 timeout -k 10 200 python bench.py --strategy $st --steps 20 > gpurun_out/bench_self_$st.log 2>&1 || { tail -20 gpurun_out/bench_self_$st.log; exit 1; }
  tail -1 gpurun_out/bench_self_$st.log
done
timeout -k 10 200 python bench.py > gpurun_out/bench_plain.log 2>&1 || { tail -20 gpurun_out/bench_plain.log; exit 1; }
tail -1 gpurun_out/bench_plain.log
