#!/bin/bash
# Round-2: pipelined DDP step (multi-cut, per-bucket all-reduce + SGD on the comm stream) —
# GPU tests, then one-GPU A/B at b32 / b256 with a timed stand-in collective (171 GB/s = 8-GPU
# ring model) and with the live single-rank RCCL communicator.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/seg
T=${TESTS:-"tests/test_gpu_model.py tests/test_gpu_rccl_self.py tests/test_gpu_resnet.py"}
timeout -k 10 600 python -u -m pytest $T -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/seg/tests.log 2>&1 || { tail -40 gpurun_out/seg/tests.log; exit 1; }
tail -2 gpurun_out/seg/tests.log
run() {  # tag, env..., -- bench args
  local tag=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 180 python bench.py --steps 60 --warmup 10 --ref-window 0 "$@" > gpurun_out/seg/$tag.log 2>&1 || { tail -5 gpurun_out/seg/$tag.log; exit 1; }
  echo "$tag $(python -c "import json; d=json.loads(open('gpurun_out/seg/$tag.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['config']['comm'], d['train_loss_mean'])")"
}
for B in 32 256; do
  run b${B}_none X=1 -- --global-batch $B
  run b${B}_emu_inline DDP_AMD_EMULATE_COMM_GBPS=171 -- --global-batch $B --segmented 0
  run b${B}_emu_seg4 DDP_AMD_EMULATE_COMM_GBPS=171 -- --global-batch $B --segmented 4
  run b${B}_emu_seg25 DDP_AMD_EMULATE_COMM_GBPS=171 -- --global-batch $B --segmented 2,5
  run b${B}_emu_seg36 DDP_AMD_EMULATE_COMM_GBPS=171 -- --global-batch $B --segmented 3,6
  run b${B}_rccl_inline DDP_AMD_RCCL_SELF=1 -- --global-batch $B --segmented 0
  run b${B}_rccl_seg4 DDP_AMD_RCCL_SELF=1 -- --global-batch $B --segmented 4
  run b${B}_rccl_seg4_bf16 DDP_AMD_RCCL_SELF=1 -- --global-batch $B --segmented 4 --grad-comm bf16
done
