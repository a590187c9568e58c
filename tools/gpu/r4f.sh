#!/bin/bash
# round 4 (XF off by default): A/B of SGD in the backward and the k-major tap-reuse dgrad at the
# four strong-scaling batches, step profiles, per-layer roofline, structure microbench
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r4f; mkdir -p $O
for CFG in 256 128 64 32; do
  for V in "base:" "nosgd:DDP_AMD_SGD_IN_BWD=0" "trdg:DDP_AMD_DGRAD_TR=1"; do
    NAME=${V%%:*}; ENVS=${V#*:}
    L=$O/b${CFG}_$NAME.log
    env $ENVS timeout -k 10 200 python bench.py --global-batch $CFG --steps 60 --warmup 10 --ref-window 0 > $L 2>&1 || { tail -5 $L; exit 1; }
    echo "b$CFG $NAME $(python -c "import json; d=json.loads(open('$L').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['train_loss_mean'])")"
  done
done
TAG=r4f BATCHES="256 32" bash tools/gpu/profile.sh || exit 1
timeout -k 10 240 python -u tools/probes/roofline.py --batch 256 32 --json $O/roofline.json > $O/roofline.log 2>&1 || { tail -5 $O/roofline.log; exit 1; }
grep totals $O/roofline.log
timeout -k 10 180 tools/probes/gemm_struct.bin 30 > $O/gemm_struct.jsonl 2>&1 || { tail -5 $O/gemm_struct.jsonl; exit 1; }
wc -l $O/gemm_struct.jsonl
