#!/bin/bash
# Which knob makes the captured ResNet-50 step corrupt its state? Runs the eager-vs-graph probe
# RUNS times per environment variant; a broken run shows graph losses pinned at ln(1000)=6.9078.
cd "$GRAFT_REPO_ROOT" || exit 2
OUT=gpurun_out/bisect
mkdir -p $OUT
for V in ${VARIANTS:-base:}; do
  NAME=${V%%:*}; ENVS=${V#*:}
  bad=0
  for R in $(seq 1 ${RUNS:-3}); do
    L=$OUT/${NAME}_r$R.log
    env ${ENVS//,/ } timeout -k 10 200 python tools/probes/resnet_graph_probe.py --steps 5 ${PROBE_ARGS:-} > $L 2>&1 || { tail -5 $L; exit 1; }
    if grep "^graph" $L | grep -q "6.90[78]"; then bad=$((bad+1)); fi
  done
  echo "$NAME broken $bad/${RUNS:-3}: $(grep '^graph' $L)"
done
