#!/bin/bash
# Reference-compatible entry points on one MI355X: part1 (single process), the three
# distributed mains at world size 1 launched reference-style (flags) and part3 under torchrun.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python part1/main.py --max-batches 45 > gpurun_out/part1.log 2>&1 || { tail -5 gpurun_out/part1.log; exit 1; }
echo "== part1"; tail -4 gpurun_out/part1.log
port=29620
for p in part2/part2a part2/part2b part3; do
  port=$((port + 1))
  timeout -k 10 240 python $p/main.py --num-nodes 1 --rank 0 --master-ip 127.0.0.1 --master-port $port \
    --max-batches 45 > gpurun_out/$(basename $p).log 2>&1 || { echo "$p failed"; tail -8 gpurun_out/$(basename $p).log; exit 1; }
  echo "== $p"; tail -4 gpurun_out/$(basename $p).log
done
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29631 part3/main.py --max-batches 45 > gpurun_out/part3_torchrun.log 2>&1 || { echo "torchrun part3 failed"; tail -8 gpurun_out/part3_torchrun.log; exit 1; }
echo "== part3 (torchrun)"; tail -4 gpurun_out/part3_torchrun.log
for p in part1 part3; do
  if [ $p = part1 ]; then
    timeout -k 10 240 python part1/main.py --graph --max-batches 45 > gpurun_out/${p}_graph.log 2>&1 || { echo "$p --graph failed"; tail -8 gpurun_out/${p}_graph.log; exit 1; }
  else
    timeout -k 10 240 python part3/main.py --graph --num-nodes 1 --rank 0 --master-ip 127.0.0.1 --master-port 29641 --max-batches 45 > gpurun_out/${p}_graph.log 2>&1 || { echo "$p --graph failed"; tail -8 gpurun_out/${p}_graph.log; exit 1; }
  fi
  echo "== $p --graph"; grep -v "amdgpu.ids\|socket.cpp" gpurun_out/${p}_graph.log | tail -5
done
