#!/bin/bash
# round 5 checkpoint: full GPU suite + smoke + default bench x2 + ResNet-50 bench + step profiles
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/${TAG:-r5x}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { grep -E "FAIL|Error" $O/gpu_tests.log | head -20; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for i in 1 2; do
  timeout -k 10 200 python bench.py > $O/bench_$i.log 2>&1 || { tail -5 $O/bench_$i.log; exit 1; }
  tail -1 $O/bench_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['ms_per_step'], d['value'], d['avg_ms_iter_1_39'], d['train_loss_mean'])"
done
cp $O/bench_2.log $O/bench_default.json
timeout -k 10 300 python bench.py --model resnet50 --steps 8 --warmup 4 --ref-window 0 > $O/resnet.log 2>&1 || { tail -5 $O/resnet.log; exit 1; }
tail -1 $O/resnet.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('resnet', d['ms_per_step'], d['value'], d['train_loss_mean'])"
TAG=${TAG:-r5x} MODEL=vgg11 BATCHES="256 32" bash tools/gpu/profile.sh && TAG=${TAG:-r5x} MODEL=resnet50 BATCHES=256 bash tools/gpu/profile.sh
# strong-scaling per-GPU shares (N = 2 / 4 / 8 of the 256 global batch)
for b in 128 64 32; do
  timeout -k 10 200 python bench.py --global-batch $b --steps 60 --warmup 10 > $O/b$b.log 2>&1 || { tail -5 $O/b$b.log; exit 1; }
  tail -1 $O/b$b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('b$b', d['ms_per_step'], d['value'])"
done
