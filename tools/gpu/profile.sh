#!/bin/bash
# rocprofv3 kernel trace (+ stats) of bench.py steps, one run per batch, summarised to markdown.
#   TAG=r3 MODEL=vgg11 BATCHES="256 32" [ENVS="A=1 B=2"] bash tools/gpu/profile.sh
# Output: gpurun_out/prof/<tag>_<model>_b<B>/ (CSV) and gpurun_out/prof/<tag>_<model>_b<B>.md
cd "$GRAFT_REPO_ROOT" || exit 2
TAG=${TAG:-prof}; MODEL=${MODEL:-vgg11}; BATCHES=${BATCHES:-"256 32"}
STEPS=20; [ "$MODEL" = resnet50 ] && STEPS=6
mkdir -p gpurun_out/prof
for B in $BATCHES; do
  N=${TAG}_${MODEL}_b$B
  D=$GRAFT_REPO_ROOT/gpurun_out/prof/$N
  (cd /tmp && export TMPDIR=/tmp && { [ -z "$ENVS" ] || export $ENVS; } && timeout -k 10 300 rocprofv3 --kernel-trace --stats \
     --output-format csv -d "$D" -o p -- python3 "$GRAFT_REPO_ROOT/bench.py" --model $MODEL \
     --global-batch $B --steps $STEPS --warmup 5 --ref-window 0 > "$D.log" 2>&1) || { tail -5 "$D.log"; exit 1; }
  P=$(ls "$D"/*/p_kernel_stats.csv 2>/dev/null | head -1); P=${P%_kernel_stats.csv}
  [ -z "$P" ] && P=$(ls "$D"/p_kernel_stats.csv | head -1 | sed 's/_kernel_stats.csv//')
  python3 tools/prof_summary.py "$P" "$N" > gpurun_out/prof/$N.md || exit 1
  grep -m1 "One training step" gpurun_out/prof/$N.md
done
