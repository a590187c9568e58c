#!/bin/bash
# One-GPU stand-in study of the multi-GPU pipelined step (engine/step.py SegmentedDDPStep): the
# collectives are timed 32-CU stand-ins at an 8-GPU all-reduce algorithm bandwidth (GBPS), the
# sharded update (--update shard16) shards as rank 0 of EMU_WORLD ranks. Per batch x cut set x
# update plan: ms/step of bench.py, PASSES interleaved passes (same box, same session).
#   BATCHES="32 64" CUTS="3,6 3,5,7" UPDATES="allreduce shard16" GBPS=171 bash tools/gpu/standin_sweep.sh
cd "$GRAFT_REPO_ROOT" || exit 2
OUT=gpurun_out/${TAG:-standin}
mkdir -p $OUT
BATCHES=${BATCHES:-"32 64 128 256"}; CUTS=${CUTS:-"3,6 3,5,7 2,5 2,4,6"}
UPDATES=${UPDATES:-"allreduce shard16"}; GBPS=${GBPS:-171}; PASSES=${PASSES:-2}
for P in $(seq 1 $PASSES); do
  for B in $BATCHES; do
    for C in $CUTS; do
      for U in $UPDATES; do
        L=$OUT/b${B}_c${C//,/-}_${U}_g${GBPS}_p$P.log
        DDP_AMD_EMULATE_COMM_GBPS=$GBPS DDP_AMD_EMULATE_WORLD=${EMU_WORLD:-8} timeout -k 10 240 \
          python bench.py --global-batch $B --steps 60 --warmup 10 --ref-window 0 --segmented $C \
          --update $U > $L 2>&1 || { tail -5 $L; exit 1; }
        echo "B=$B cuts=$C $U g=$GBPS p$P $(python -c "import json; d=json.loads(open('$L').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['comm_plan'].get('update_plan', {}).get('update'))")"
      done
    done
  done
done
