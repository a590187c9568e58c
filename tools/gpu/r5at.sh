#!/bin/bash
# round 5: knob re-check at the N = 2 / 4 per-GPU shares (b128 / b64) on the current kernels —
# environment only, no rebuild; baseline runs interleaved with the variants
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r5at; mkdir -p $O
run() {  # $1 = batch, $2 = label, rest = env assignments
  local b=$1 l=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --global-batch $b --steps 60 --warmup 10 > $O/b${b}_$l.log 2>&1 || { tail -5 $O/b${b}_$l.log; exit 1; }
  tail -1 $O/b${b}_$l.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('b$b $l', d['ms_per_step'])"
}
for b in 128 64; do
  run $b base1 X=1
  run $b poolmax128 DDP_AMD_FUSE_BN_IN_POOL_MAX_BATCH=128
  run $b fusehw16 DDP_AMD_BN_BWD_FUSE_MAX_HW=16
  run $b fusehw256 DDP_AMD_BN_BWD_FUSE_MAX_HW=256
  run $b base2 X=1
  run $b local5 DDP_AMD_BN_BWD_LOCAL_LOADS=5
  run $b local12 DDP_AMD_BN_BWD_LOCAL_LOADS=12
  run $b rows256 DDP_AMD_BN_FUSE_MAX_ROWS=256
  run $b fold0 DDP_AMD_BN_FOLD_BWD_MB=0
  run $b fold96 DDP_AMD_BN_FOLD_BWD_MB=96
  run $b base3 X=1
done
