#!/bin/bash
# round 4: after removing the apply-free BN backward (XF) and the tap-reuse dgrad: full GPU
# suite, bench A/B of the tile-order knob (DDP_AMD_TILE_ORDER=n) at b256/b32, ResNet-50 step
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r4m; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { grep -E "FAIL|Error" $O/gpu_tests.log | head -20; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for P in 1 2; do
for CFG in 256 32; do
  for V in "base:" "ordn:DDP_AMD_TILE_ORDER=n"; do
    NAME=${V%%:*}; ENVS=${V#*:}
    L=$O/b${CFG}_${NAME}_p$P.log
    env $ENVS timeout -k 10 200 python bench.py --global-batch $CFG --steps 60 --warmup 10 --ref-window 0 > $L 2>&1 || { tail -5 $L; exit 1; }
    echo "b$CFG $NAME p$P $(python -c "import json; d=json.loads(open('$L').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['train_loss_mean'])")"
  done
done
done
for V in "base:" "ordn:DDP_AMD_TILE_ORDER=n"; do
  NAME=${V%%:*}; ENVS=${V#*:}
  L=$O/resnet_${NAME}.log
  env $ENVS timeout -k 10 300 python bench.py --model resnet50 --steps 8 --warmup 4 --ref-window 0 > $L 2>&1 || { tail -5 $L; exit 1; }
  echo "resnet50 $NAME $(python -c "import json; d=json.loads(open('$L').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['train_loss_mean'])")"
done
