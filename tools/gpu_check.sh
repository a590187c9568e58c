#!/bin/bash
# GPU-box check: numerics tests, 1-GPU bench, kernel-trace profile.
# Usage (from the container): gpurun --timeout 900 -- bash tools/gpu_check.sh [tests|bench|prof]...
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
steps="${@:-tests bench prof}"
ok_or_stop() {  # continue only after a clean exit or an ordinary test failure
  local rc=$1 what=$2
  echo "$what rc=$rc"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "stopping after $what rc=$rc"; exit "$rc"; fi
}
for s in $steps; do
  case $s in
    tests)
      timeout -k 10 600 python -m pytest tests -q -m gpu -p no:cacheprovider -rA > gpurun_out/pytest_gpu.log 2>&1
      rc=$?; grep -E "passed|failed|error|rel err" gpurun_out/pytest_gpu.log | tail -15; ok_or_stop $rc pytest ;;
    bench)
      timeout -k 10 300 python bench.py --steps 40 --warmup 10 > gpurun_out/bench1.log 2>&1
      rc=$?; tail -3 gpurun_out/bench1.log; ok_or_stop $rc bench ;;
    benchatomic)  # split-K weight gradients with fp32 atomics
      DDP_AMD_WGRAD_ATOMIC=1 timeout -k 10 300 python bench.py --steps 40 --warmup 10 > gpurun_out/bench_atomic.log 2>&1
      rc=$?; tail -1 gpurun_out/bench_atomic.log; ok_or_stop $rc bench_atomic ;;
    benchresnet)
      timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/bench_resnet.log 2>&1
      rc=$?; tail -1 gpurun_out/bench_resnet.log; ok_or_stop $rc bench_resnet ;;
    profresnet)
      root="$GRAFT_REPO_ROOT"
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats \
          --output-format csv -d "$root/gpurun_out/prof_resnet" -o resnet -- \
          python3 "$root/bench.py" --model resnet50 --steps 6 --warmup 3 > "$root/gpurun_out/prof_resnet.log" 2>&1)
      rc=$?; tail -1 gpurun_out/prof_resnet.log; ok_or_stop $rc prof_resnet ;;
    convbench)
      timeout -k 10 300 python tools/conv_bench.py --model vgg11 --json gpurun_out/conv_vgg.json > gpurun_out/conv_vgg.log 2>&1
      rc=$?; tail -1 gpurun_out/conv_vgg.log; ok_or_stop $rc convbench_vgg
      timeout -k 10 300 python tools/conv_bench.py --model resnet50 --json gpurun_out/conv_resnet.json > gpurun_out/conv_resnet.log 2>&1
      rc=$?; tail -1 gpurun_out/conv_resnet.log; ok_or_stop $rc convbench_resnet ;;
    convbenchp)  # persistent conv grids
      DDP_AMD_CONV_PERSISTENT=1 timeout -k 10 300 python tools/conv_bench.py --model vgg11 --json gpurun_out/conv_vgg_p.json > gpurun_out/conv_vgg_p.log 2>&1
      rc=$?; tail -1 gpurun_out/conv_vgg_p.log; ok_or_stop $rc convbench_vgg_p
      DDP_AMD_CONV_PERSISTENT=1 timeout -k 10 300 python tools/conv_bench.py --model resnet50 --json gpurun_out/conv_resnet_p.json > gpurun_out/conv_resnet_p.log 2>&1
      rc=$?; tail -1 gpurun_out/conv_resnet_p.log; ok_or_stop $rc convbench_resnet_p ;;
    bench8w)  # weak-scaling point and eager (no graph) comparison
      timeout -k 10 300 python bench.py --steps 40 --warmup 10 --no-graph > gpurun_out/bench_eager.log 2>&1
      rc=$?; tail -1 gpurun_out/bench_eager.log; ok_or_stop $rc bench_eager ;;
    prof)
      root="$GRAFT_REPO_ROOT"
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats \
          --output-format csv -d "$root/gpurun_out/prof" -o vgg11 -- \
          python3 "$root/bench.py" --steps 20 --warmup 5 > "$root/gpurun_out/prof.log" 2>&1)
      rc=$?; tail -2 gpurun_out/prof.log; ok_or_stop $rc prof
      find gpurun_out/prof -name "*kernel_stats.csv" | head -3 ;;
  esac
done
exit 0
