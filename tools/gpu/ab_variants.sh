#!/bin/bash
# Same-session A/B of (native build, conv tuning table) pairs, benches interleaved over passes.
#   VARIANTS="r5:ab_so/_native_r5.so:ab_so/conv_tuning_r5.json cur::" CFGS="vgg11:256 vgg11:32" \
#       PASSES=2 bash tools/gpu/ab_variants.sh
# An empty .so / table field means the in-tree one (an empty DDP_AMD_CONV_TUNING_FILE would
# load NO table, so the variable is only set when a table is named).
cd "$GRAFT_REPO_ROOT" || exit 2
OUT=gpurun_out/ab_var
mkdir -p $OUT
VARIANTS=${VARIANTS:-"cur::"}
CFGS=${CFGS:-"vgg11:256 vgg11:32"}
for P in $(seq 1 ${PASSES:-2}); do
  for CFG in $CFGS; do
    M=${CFG%%:*}; B=${CFG##*:}; S=60; [ $M = resnet50 ] && S=12
    for V in $VARIANTS; do
      NAME=${V%%:*}; REST=${V#*:}; SO=${REST%%:*}; TAB=${REST#*:}
      L=$OUT/${M}_b${B}_${NAME}_p$P.log
      ENVS=()
      [ -n "$SO" ] && ENVS+=("DDP_AMD_NATIVE_PATH=$SO")
      [ -n "$TAB" ] && ENVS+=("DDP_AMD_CONV_TUNING_FILE=$TAB")
      env "${ENVS[@]}" timeout -k 10 240 python bench.py --model $M --global-batch $B --steps $S \
          --warmup 10 --ref-window 0 > $L 2>&1 || { tail -5 $L; exit 1; }
      echo "$M B=$B $NAME p$P $(python -c "import json; d=json.loads(open('$L').read().strip().splitlines()[-1]); print(d['ms_per_step'])")"
    done
  done
done
