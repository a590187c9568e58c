#!/bin/bash
# round 5: backward contention under a paced, traffic-carrying stand-in collective
# (tools/pipeline_probe.py --passes N: the stand-in streams its bucket N times over its
# modelled time instead of once at its start)
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r5j; mkdir -p $O
for b in 32 256; do
  for u in shard16 allreduce; do
    for p in 1 4; do
      timeout -k 10 240 python -u tools/pipeline_probe.py --batch $b --cuts 3,6 --update $u --passes $p \
        > $O/probe_b${b}_${u}_p${p}.log 2>&1 || { tail -20 $O/probe_b${b}_${u}_p${p}.log; exit 1; }
      grep contention $O/probe_b${b}_${u}_p${p}.log | sed "s/^/b$b $u p$p: /"
    done
  done
done
