#!/bin/bash
# Environment-knob A/B on the default bench (VGG-11 b256, 1 GPU): bash tools/gpu_knob_sweep.sh
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
run() {
  local label=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 200 --warmup 20 > gpurun_out/knob.log 2>&1 || { echo "$label FAILED"; tail -5 gpurun_out/knob.log; exit 1; }
  echo "$label $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/knob.log)"
}
run default DDP_AMD_X=0
run persistent DDP_AMD_CONV_PERSISTENT=1
run bwdblocks512 DDP_AMD_BN_BWD_BLOCKS=512
run bwdblocks2048 DDP_AMD_BN_BWD_BLOCKS=2048
run bnlastblock DDP_AMD_BN_LAST_BLOCK=1
run default2 DDP_AMD_X=0
