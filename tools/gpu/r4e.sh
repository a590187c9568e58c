#!/bin/bash
# round 4: PMC passes over one VGG-11 b256 step; ResNet-50 b256 with / without the apply-free BN
# backward + its step profile; ResNet-50 1x1 convolutions vs hipBLASLt; bench warm-up check
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r4e; mkdir -p $O
for V in 0 1; do
  DDP_AMD_BN_BWD_XF=$V timeout -k 10 300 python bench.py --model resnet50 --steps 8 --warmup 4 --ref-window 0 > $O/resnet_xf$V.log 2>&1 || { tail -5 $O/resnet_xf$V.log; exit 1; }
  echo "resnet50 b256 xf=$V $(python -c "import json; d=json.loads(open('$O/resnet_xf$V.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['train_loss_mean'])")"
done
TAG=r4e MODEL=resnet50 BATCHES="256" bash tools/gpu/profile.sh || exit 1
timeout -k 10 300 python -u tools/probes/resnet_1x1_table.py --batch 256 --json $O/resnet_1x1.json > $O/resnet_1x1.log 2>&1 || { tail -5 $O/resnet_1x1.log; exit 1; }
tail -1 $O/resnet_1x1.log
for SW in "20 5" "20 30" "60 10" "20 5"; do set -- $SW
  timeout -k 10 200 python bench.py --steps $1 --warmup $2 > $O/bench_s$1_w$2.log 2>&1 || { tail -5 $O/bench_s$1_w$2.log; exit 1; }
  echo "steps=$1 warmup=$2 $(python -c "import json; d=json.loads(open('$O/bench_s$1_w$2.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['avg_ms_iter_1_39'])")"
done
bash tools/gpu/pmc.sh > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
python tools/pmc_summary.py gpurun_out/pmc > $O/pmc_b256.md && head -3 $O/pmc_b256.md
