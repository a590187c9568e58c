#!/bin/bash
# Round-2: ZeRO-1 sharded update + trajectory test + bench A/B (live single-rank RCCL)
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/zero
timeout -k 10 600 python -u -m pytest ${ZT:-tests/test_gpu_rccl_self.py tests/test_gpu_model.py::test_vgg11_20_step_trajectory_matches_cpu_fp32_oracle} -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/zero/tests.log 2>&1 || { tail -40 gpurun_out/zero/tests.log; exit 1; }
grep -E "passed|failed|cpu fp32|gpu bf16|cosine" gpurun_out/zero/tests.log | tail -6
for B in 32 256; do
  for V in rep zero; do
    Z=""; [ $V = zero ] && Z="--zero"
    DDP_AMD_RCCL_SELF=1 timeout -k 10 180 python bench.py --global-batch $B --steps 60 --warmup 10 --ref-window 0 --segmented 3,6 $Z > gpurun_out/zero/b${B}_$V.log 2>&1 || { tail -5 gpurun_out/zero/b${B}_$V.log; exit 1; }
    echo "B=$B $V $(python -c "import json; d=json.loads(open('gpurun_out/zero/b${B}_$V.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['train_loss_mean'])")"
  done
done
