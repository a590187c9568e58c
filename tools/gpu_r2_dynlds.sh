#!/bin/bash
# dynamic LDS ring sized to the k-steps a work item uses: kernel tests, per-conv probe, benches
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/dyn
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/dyn/kernels.log 2>&1 || { tail -30 gpurun_out/dyn/kernels.log; exit 1; }
tail -1 gpurun_out/dyn/kernels.log
timeout -k 10 150 python -u tools/stat_probe.py > gpurun_out/dyn/probe_resnet.log 2>&1 || { tail gpurun_out/dyn/probe_resnet.log; exit 1; }
cat gpurun_out/dyn/probe_resnet.log
for CFG in "vgg11 256" "vgg11 32" "resnet50 256"; do
  set -- $CFG; M=$1; B=$2; S=60; [ $M = resnet50 ] && S=20
  L=gpurun_out/dyn/${M}_b$B.log
  timeout -k 10 240 python bench.py --model $M --global-batch $B --steps $S --warmup 10 --ref-window 0 > $L 2>&1 || { tail -5 $L; exit 1; }
  echo "$M B=$B $(python -c "import json; d=json.loads(open('$L').read().strip().splitlines()[-1]); print(d['ms_per_step'], d.get('train_loss_mean'))")"
done
[ -n "$WITH_PMC" ] && PMC_SETS=insts bash tools/gpu_r2_pmc64.sh
true
