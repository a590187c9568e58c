#!/bin/bash
# round 5: captured-memset ordering probe; default bench x2; step profiles b256 / b32
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r5g; mkdir -p $O
timeout -k 10 300 python tools/probes/memset_graph_probe.py > $O/memset.json 2> $O/memset.err || { tail -20 $O/memset.err; exit 1; }
tail -1 $O/memset.json
for i in 1 2; do
  timeout -k 10 200 python bench.py > $O/bench_$i.log 2>&1 || { tail -5 $O/bench_$i.log; exit 1; }
  tail -1 $O/bench_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['ms_per_step'], d['value'], d['avg_ms_iter_1_39'], d['train_loss_mean'])"
done
TAG=r5g BATCHES="256 32" bash tools/gpu/profile.sh
