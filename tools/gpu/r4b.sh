#!/bin/bash
# round 4: apply-free BN backward (XF) — kernel tests, model tests, then benches + profiles
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r4b; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "xf or bn_act_fwd_bwd" -x -v --timeout 120 --timeout-method thread > $O/k1.log 2>&1 || { tail -40 $O/k1.log; exit 1; }
tail -1 $O/k1.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -x -v --timeout 300 --timeout-method thread > $O/k2.log 2>&1 || { tail -60 $O/k2.log; exit 1; }
tail -1 $O/k2.log
grep -A12 "lr01_headline" $O/k2.log | grep -E "^(fused|emu|fp32|k0)" | head -12
for B in 256 32 64 128; do
  timeout -k 10 200 python bench.py --global-batch $B --steps 60 --warmup 10 --ref-window 0 > $O/bench_b$B.log 2>&1 || { tail -5 $O/bench_b$B.log; exit 1; }
  echo "b$B $(python -c "import json; d=json.loads(open('$O/bench_b$B.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['train_loss_mean'])")"
  DDP_AMD_BN_BWD_XF=0 timeout -k 10 200 python bench.py --global-batch $B --steps 60 --warmup 10 --ref-window 0 > $O/bench_b${B}_noxf.log 2>&1 || { tail -5 $O/bench_b${B}_noxf.log; exit 1; }
  echo "b$B noxf $(python -c "import json; d=json.loads(open('$O/bench_b${B}_noxf.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['train_loss_mean'])")"
done
TAG=r4b BATCHES="256 32" bash tools/gpu/profile.sh
timeout -k 10 300 python -u tools/probes/roofline.py --batch 256 32 --json $O/roofline.json > $O/roofline.log 2>&1 || { tail -5 $O/roofline.log; exit 1; }
grep totals $O/roofline.log
