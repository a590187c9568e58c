#!/bin/bash
# Split-K fixup (in-kernel last-block reduction) vs finish kernels: GPU tests + same-box A/B.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { grep -E "FAIL|Error|error" gpurun_out/gputests.log | head -20; tail -5 gpurun_out/gputests.log; exit 1; }
tail -1 gpurun_out/gputests.log
b() { local label=$1 envs=$2; shift 2
  timeout -k 10 200 env $envs python bench.py --steps 60 --warmup 10 "$@" > gpurun_out/fx.log 2>&1 || { tail -5 gpurun_out/fx.log; exit 1; }
  echo "| $label | $envs $* | $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/fx.log | cut -d' ' -f2) |"; }
for i in 1 2 3; do
b fixup "DDP_AMD_SPLITK_FIXUP=1"
b finish "DDP_AMD_SPLITK_FIXUP=0"
done
b fixup_resnet "DDP_AMD_SPLITK_FIXUP=1" --model resnet50 --steps 10 --warmup 3
b finish_resnet "DDP_AMD_SPLITK_FIXUP=0" --model resnet50 --steps 10 --warmup 3
