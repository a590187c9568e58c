#!/bin/bash
# round 4: SGD-in-backward kernel test + trajectory; same-session A/B (SGD in backward, tile
# order); ResNet-50 with the apply-free BN backward; PMC passes; structure microbench; probes
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r4c; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "sgd_in_backward or bwd_pair" -x -v --timeout 120 --timeout-method thread > $O/k1.log 2>&1 || { tail -40 $O/k1.log; exit 1; }
tail -1 $O/k1.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_model.py -k "graph_step_equals_eager or trajectory or lr01" -x -v --timeout 300 --timeout-method thread > $O/k2.log 2>&1 || { tail -40 $O/k2.log; exit 1; }
tail -1 $O/k2.log
NOTEST=1 VARIANTS="base: nosgd:DDP_AMD_SGD_IN_BWD=0 tn:DDP_AMD_TILE_ORDER=n" CFGS="vgg11:256 vgg11:32" bash tools/gpu/ab_env.sh || exit 1
for SW in "20 5" "20 30" "60 10" "20 5"; do set -- $SW
  timeout -k 10 200 python bench.py --steps $1 --warmup $2 > $O/bench_s$1_w$2.log 2>&1 || { tail -5 $O/bench_s$1_w$2.log; exit 1; }
  echo "steps=$1 warmup=$2 $(python -c "import json; d=json.loads(open('$O/bench_s$1_w$2.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['avg_ms_iter_1_39'])")"
done
for V in 1 0; do
  DDP_AMD_BN_BWD_XF=$V timeout -k 10 300 python bench.py --model resnet50 --steps 8 --warmup 4 --ref-window 0 > $O/resnet_xf$V.log 2>&1 || { tail -5 $O/resnet_xf$V.log; exit 1; }
  echo "resnet50 b256 xf=$V $(python -c "import json; d=json.loads(open('$O/resnet_xf$V.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['train_loss_mean'])")"
done
timeout -k 10 180 tools/probes/gemm_struct.bin 50 > $O/gemm_struct.jsonl 2>&1 || { tail -5 $O/gemm_struct.jsonl; exit 1; }
TAG=r4c BATCHES="256 32" bash tools/gpu/profile.sh || exit 1
bash tools/gpu/pmc.sh > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
python tools/pmc_summary.py gpurun_out/pmc > $O/pmc_b256.md
TAG=r4c MODEL=resnet50 BATCHES="256" bash tools/gpu/profile.sh || exit 1
timeout -k 10 300 python -u tools/probes/resnet_1x1_table.py --batch 256 --json $O/resnet_1x1.json > $O/resnet_1x1.log 2>&1 || { tail -5 $O/resnet_1x1.log; exit 1; }
