#!/bin/bash
# Scaling report on ONE node with >= 8 MI355X (not runnable on a 1-GPU box):
#   1. the all-reduce bus-bandwidth table for 2/4/8 ranks (fp32 and bf16) -> the bucket-sizing
#      table parallel/comm_tuning.json ("measured" rows replace the latency/bandwidth model);
#   2. every strategy (part3 DDP, part2b all_reduce, part2a gather/scatter and
#      gather/broadcast) at 1/2/4/8 GPUs, the reference's strong-scaling protocol (global batch
#      256 split int(256/N) per GPU, the bench default) and weak scaling (--per-gpu-batch 256).
# Every multi-rank run is self-launched (bench.py / comm_bench.py --gpus N spawn one process per
# GPU; no torchrun needed). One JSON line per run in gpurun_out/scale_sweep.jsonl; summarise
# with python tools/scale_report.py.
#   bash tools/scale_sweep.sh [max_gpus] [--no-table]
cd "$(dirname "$0")/.." || exit 2
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
out=gpurun_out/scale_sweep.jsonl
: > "$out"
max=${1:-8}
if [ "$2" != "--no-table" ]; then
  for n in 2 4 8; do
    [ $n -gt "$max" ] && continue
    for dt in fp32 bf16; do
      timeout -k 10 600 python tools/comm_bench.py --gpus $n --dtype $dt --write-table \
        > gpurun_out/comm_bench_${n}_$dt.jsonl 2> gpurun_out/comm_bench_${n}_$dt.err \
        || { echo "comm_bench n=$n $dt failed"; tail -3 gpurun_out/comm_bench_${n}_$dt.err; exit 1; }
      echo "comm table n=$n $dt: $(tail -1 gpurun_out/comm_bench_${n}_$dt.jsonl)"
    done
  done
fi
for strat in ddp allreduce gather_scatter gather_broadcast; do
  for mode in strong weak; do
    extra=""; [ $mode = weak ] && extra="--per-gpu-batch 256"
    for n in 1 2 4 8; do
      [ $n -gt "$max" ] && continue
      timeout -k 10 600 python bench.py --gpus $n --steps 40 --warmup 10 \
        --strategy $strat $extra --json-out gpurun_out/scale_last.json > gpurun_out/scale_last.log 2>&1
      rc=$?
      if [ $rc -ne 0 ]; then echo "strategy=$strat n=$n $mode rc=$rc"; tail -3 gpurun_out/scale_last.log; exit $rc; fi
      cat gpurun_out/scale_last.json >> "$out"
      echo "strategy=$strat n=$n $mode $(grep -o '"value": [0-9.]*' gpurun_out/scale_last.json)"
    done
  done
done
