#!/bin/bash
# Reference-compatible mains on one MI355X, two passes in alternating order (measurement
# hygiene: eager per-iteration times at world 1, where the 2A/2B syncs are no-ops)
cd "$GRAFT_REPO_ROOT" || exit 2
export HSA_ENABLE_IPC_MODE_LEGACY=0
port=29700
for pass in 1 2; do
  mkdir -p gpurun_out/mains/p$pass
  order="part1 part2/part2a part2/part2b part3"
  [ $pass = 2 ] && order="part3 part2/part2b part2/part2a part1"
  for p in $order; do
    port=$((port + 1))
    name=$(basename $p)
    if [ $p = part1 ]; then
      timeout -k 10 240 python part1/main.py --max-batches 45 > gpurun_out/mains/p$pass/$name.log 2>&1 || { tail -5 gpurun_out/mains/p$pass/$name.log; exit 1; }
    else
      timeout -k 10 240 python $p/main.py --num-nodes 1 --rank 0 --master-ip 127.0.0.1 --master-port $port --max-batches 45 > gpurun_out/mains/p$pass/$name.log 2>&1 || { tail -8 gpurun_out/mains/p$pass/$name.log; exit 1; }
    fi
    echo "pass $pass $name $(grep 'Average time' gpurun_out/mains/p$pass/$name.log)"
  done
  for p in part1 part3; do
    port=$((port + 1))
    if [ $p = part1 ]; then
      timeout -k 10 240 python part1/main.py --graph --max-batches 45 > gpurun_out/mains/p$pass/${p}_graph.log 2>&1 || exit 1
    else
      timeout -k 10 240 python part3/main.py --graph --num-nodes 1 --rank 0 --master-ip 127.0.0.1 --master-port $port --max-batches 45 > gpurun_out/mains/p$pass/${p}_graph.log 2>&1 || exit 1
    fi
    echo "pass $pass $p --graph $(grep 'Average time' gpurun_out/mains/p$pass/${p}_graph.log)"
  done
done
# BN-backward in-launch finalize (last block) at the strong-scaling batches
for B in 32 64; do
  for V in 0 1; do
    DDP_AMD_BN_LAST_BLOCK=$V timeout -k 10 120 python bench.py --global-batch $B --steps 100 --warmup 10 --ref-window 0 > gpurun_out/mains/lb_b${B}_$V.log 2>&1 || exit 1
    echo "B=$B last_block=$V $(tail -1 gpurun_out/mains/lb_b${B}_$V.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
  done
done
