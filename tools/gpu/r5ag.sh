#!/bin/bash
# round 5: kernel-level comparison of the session-start tree (_oldtree/) and the current tree,
# VGG-11 b256, rocprofv3 kernel trace of each (same box)
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/prof
for t in old new; do
  if [ $t = old ]; then D=$GRAFT_REPO_ROOT/_oldtree; else D=$GRAFT_REPO_ROOT; fi
  P=$GRAFT_REPO_ROOT/gpurun_out/prof/r5ag_$t
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$P" -o p -- python3 "$D/bench.py" --steps 20 --warmup 5 --ref-window 0 > "$P.log" 2>&1) || { tail -5 "$P.log"; exit 1; }
  F=$(ls "$P"/*/p_kernel_stats.csv 2>/dev/null | head -1); F=${F%_kernel_stats.csv}
  [ -z "$F" ] && F=$(ls "$P"/p_kernel_stats.csv | head -1 | sed 's/_kernel_stats.csv//')
  python3 tools/prof_summary.py "$F" "r5ag_$t" > gpurun_out/prof/r5ag_$t.md || exit 1
  grep -m1 "One training step" gpurun_out/prof/r5ag_$t.md
done
