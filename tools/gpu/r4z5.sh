#!/bin/bash
# round 4: knob re-sweep on the strong-scaling shares (two passes per setting)
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r4z5; mkdir -p $O
run() {  # name batch env...
  local n=$1 B=$2; shift 2
  timeout -k 10 200 env "$@" python bench.py --global-batch $B --steps 60 --warmup 10 --ref-window 0 > $O/$n.log 2>&1 || { tail -5 $O/$n.log; exit 1; }
  echo "$n $(tail -1 $O/$n.log | grep -oE '"ms_per_step": [0-9.]+')"
}
for p in 1 2; do
for B in 128 64 32; do
  run b${B}_base_$p $B X=1
  run b${B}_items2048_$p $B DDP_AMD_BWD_PAIR_ITEMS=2048
  run b${B}_items512_$p $B DDP_AMD_BWD_PAIR_ITEMS=512
  run b${B}_poolin_$p $B DDP_AMD_FUSE_BN_IN_POOL_MAX_BATCH=128
  run b${B}_rows256_$p $B DDP_AMD_BN_FUSE_MAX_ROWS=256
done; done
