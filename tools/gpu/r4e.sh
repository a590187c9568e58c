#!/bin/bash
# round 4: where the GEMM time goes — per-layer roofline vs hipBLASLt, main-loop structure
# microbench, PMC passes over one b256 step, ResNet-50 with the apply-free BN backward
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r4e; mkdir -p $O
timeout -k 10 240 python -u tools/probes/roofline.py --batch 256 32 --json $O/roofline.json > $O/roofline.log 2>&1 || { tail -5 $O/roofline.log; exit 1; }
grep totals $O/roofline.log
timeout -k 10 180 tools/probes/gemm_struct.bin 30 > $O/gemm_struct.jsonl 2>&1 || { tail -5 $O/gemm_struct.jsonl; exit 1; }
wc -l $O/gemm_struct.jsonl
bash tools/gpu/pmc.sh > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
python tools/pmc_summary.py gpurun_out/pmc > $O/pmc_b256.md && head -3 $O/pmc_b256.md
for V in 1 0; do
  DDP_AMD_BN_BWD_XF=$V timeout -k 10 300 python bench.py --model resnet50 --steps 8 --warmup 4 --ref-window 0 > $O/resnet_xf$V.log 2>&1 || { tail -5 $O/resnet_xf$V.log; exit 1; }
  echo "resnet50 b256 xf=$V $(python -c "import json; d=json.loads(open('$O/resnet_xf$V.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['train_loss_mean'])")"
done
