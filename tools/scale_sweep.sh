#!/bin/bash
# Scaling report on ONE node with >= 8 MI355X (not runnable on a 1-GPU box): every strategy
# (part3 DDP, part2b all_reduce, part2a gather/scatter and gather/broadcast) at 1/2/4/8 GPUs,
# the reference's strong-scaling protocol (global batch 256 split int(256/N) per GPU, the bench
# default) and weak scaling (--per-gpu-batch 256). One JSON line per run in
# gpurun_out/scale_sweep.jsonl; summarise with python tools/scale_report.py.
#   bash tools/scale_sweep.sh [max_gpus]
cd "$(dirname "$0")/.." || exit 2
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
out=gpurun_out/scale_sweep.jsonl
: > "$out"
max=${1:-8}
port=29600
for strat in ddp allreduce gather_scatter gather_broadcast; do
  for mode in strong weak; do
    extra=""; [ $mode = weak ] && extra="--per-gpu-batch 256"
    for n in 1 2 4 8; do
      [ $n -gt "$max" ] && continue
      port=$((port + 1))
      timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
        --master-addr 127.0.0.1 --master-port $port bench.py --gpus $n --steps 40 --warmup 10 \
        --strategy $strat $extra --json-out gpurun_out/scale_last.json > gpurun_out/scale_last.log 2>&1
      rc=$?
      if [ $rc -ne 0 ]; then echo "strategy=$strat n=$n $mode rc=$rc"; tail -3 gpurun_out/scale_last.log; exit $rc; fi
      cat gpurun_out/scale_last.json >> "$out"
      echo "strategy=$strat n=$n $mode $(grep -o '"value": [0-9.]*' gpurun_out/scale_last.json)"
    done
  done
done
