#!/bin/bash
# round 4: ResNet-50 b256 with the apply-free BN backward (bench + XF A/B + step profile), PMC
# passes over one VGG-11 b256 step, VGG-11 b64/b128 step profiles
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r4c; mkdir -p $O
for V in 1 0; do
  DDP_AMD_BN_BWD_XF=$V timeout -k 10 300 python bench.py --model resnet50 --steps 8 --warmup 4 --ref-window 0 > $O/resnet_xf$V.log 2>&1 || { tail -5 $O/resnet_xf$V.log; exit 1; }
  echo "resnet50 b256 xf=$V $(python -c "import json; d=json.loads(open('$O/resnet_xf$V.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['train_loss_mean'])")"
done
TAG=r4c MODEL=resnet50 BATCHES="256" bash tools/gpu/profile.sh || exit 1
TAG=r4c BATCHES="128 64" bash tools/gpu/profile.sh || exit 1
bash tools/gpu/pmc.sh > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
python tools/pmc_summary.py gpurun_out/pmc > $O/pmc_b256.md && grep -c conv $O/pmc_b256.md
NOTEST=1 VARIANTS="m: n:DDP_AMD_TILE_ORDER=n" CFGS="vgg11:256 vgg11:32 resnet50:256" bash tools/gpu/ab_env.sh
timeout -k 10 180 tools/probes/gemm_struct.bin 50 > $O/gemm_struct.jsonl 2>&1 || { tail -5 $O/gemm_struct.jsonl; exit 1; }
timeout -k 10 300 python -u tools/probes/resnet_1x1_table.py --batch 256 --json $O/resnet_1x1.json > $O/resnet_1x1.log 2>&1 || { tail -5 $O/resnet_1x1.log; exit 1; }
