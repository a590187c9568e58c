#!/bin/bash
# Same-session comparison: plain PyTorch-ROCm (eager + torch.cuda.graph) vs this framework's
# bench.py on the same configs. Output: gpurun_out/baseline/*.jsonl
cd "$GRAFT_REPO_ROOT" || exit 2
OUT=gpurun_out/baseline
mkdir -p $OUT
timeout -k 10 400 python -u tools/torch_baseline.py --model vgg11 --batch 256 32 --steps 50 > $OUT/torch_vgg11.jsonl 2>$OUT/torch_vgg11.err || { tail -5 $OUT/torch_vgg11.err; exit 1; }
cat $OUT/torch_vgg11.jsonl
timeout -k 10 400 python -u tools/torch_baseline.py --model resnet50 --batch 256 --steps 10 --warmup 3 > $OUT/torch_resnet50.jsonl 2>$OUT/torch_resnet50.err || { tail -5 $OUT/torch_resnet50.err; exit 1; }
cat $OUT/torch_resnet50.jsonl
for CFG in vgg11:256 vgg11:32 resnet50:256; do
  M=${CFG%%:*}; B=${CFG##*:}; S=60; [ $M = resnet50 ] && S=20
  timeout -k 10 300 python bench.py --model $M --global-batch $B --steps $S --warmup 10 --ref-window 0 --json-out $OUT/ours_${M}_b$B.json > $OUT/ours_${M}_b$B.log 2>&1 || { tail -5 $OUT/ours_${M}_b$B.log; exit 1; }
  echo "ours $M b$B $(python -c "import json; d=json.load(open('$OUT/ours_${M}_b$B.json')); print(d['ms_per_step'], d['value'])")"
done
