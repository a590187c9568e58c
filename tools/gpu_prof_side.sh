#!/bin/bash
# kernel-trace of the captured VGG step with the backward side stream on, plus strategy A/B
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
root="$GRAFT_REPO_ROOT"
for st in allreduce ddp; do
  DDP_AMD_BWD_STREAMS=1 timeout -k 10 200 python bench.py --steps 30 --warmup 5 --strategy $st > gpurun_out/side_$st.log 2>&1 || exit $?
  echo "side=1 strategy=$st $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/side_$st.log)"
done
(cd /tmp && export TMPDIR=/tmp && DDP_AMD_BWD_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace \
   --output-format csv -d "$root/gpurun_out/prof_side" -o side -- \
   python3 "$root/bench.py" --steps 8 --warmup 3 > "$root/gpurun_out/prof_side.log" 2>&1) || exit $?
f=$(find gpurun_out/prof_side -name "*kernel_trace.csv" | head -1)
python tools/timeline.py "${f%_kernel_trace.csv}" > gpurun_out/timeline_side.txt
tail -3 gpurun_out/timeline_side.txt
exit 0
