#!/bin/bash
# one GPU, no collective: does the pipelined step (per-bucket SGD on the comm stream under the
# earlier backward) beat the single graph?
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/n1seg
for B in 256 32; do
  for C in 0 3,6 2,5 2,4,6 1,3,5; do
    for rep in 1 2; do
      timeout -k 10 120 python bench.py --global-batch $B --steps 100 --warmup 10 --ref-window 0 --segmented $C > gpurun_out/n1seg/b${B}_${C//,/-}_$rep.log 2>&1 || { tail -5 gpurun_out/n1seg/b${B}_${C//,/-}_$rep.log; exit 1; }
      echo "B=$B cuts=$C rep=$rep $(tail -1 gpurun_out/n1seg/b${B}_${C//,/-}_$rep.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
    done
  done
done
