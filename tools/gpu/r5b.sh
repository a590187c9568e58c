#!/bin/bash
# round 5: pipelined-step timeline probes (stand-in collectives), b32 / b64
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r5b; mkdir -p $O
for cfg in "32 3,6 shard16" "32 3,5,7 allreduce" "32 3,5,7 shard16" "64 3,6 shard16"; do
  set -- $cfg
  timeout -k 10 120 python tools/pipeline_probe.py --batch $1 --cuts $2 --update $3 > $O/probe_b$1_${2//,/-}_$3.md 2>&1 || { tail -20 $O/probe_b$1_${2//,/-}_$3.md; exit 1; }
  head -30 $O/probe_b$1_${2//,/-}_$3.md | grep -v "^{"
done
