#!/bin/bash
# A/B of the conv LDS ring depth policy: per-layer conv bench + full bench for 2/3/4 stages.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
for st in 2 3 4; do
  DDP_AMD_CONV_STAGES=$st timeout -k 10 200 python tools/conv_bench.py --model vgg11 --json gpurun_out/conv_vgg_s$st.json > gpurun_out/conv_vgg_s$st.log 2>&1
  rc=$?; echo "stages=$st convbench rc=$rc $(tail -1 gpurun_out/conv_vgg_s$st.log)"
  [ $rc -ne 0 ] && exit $rc
  DDP_AMD_CONV_STAGES=$st timeout -k 10 200 python bench.py --steps 40 --warmup 10 > gpurun_out/bench_s$st.log 2>&1
  rc=$?; echo "stages=$st bench rc=$rc $(tail -1 gpurun_out/bench_s$st.log | cut -c1-200)"
  [ $rc -ne 0 ] && exit $rc
done
DDP_AMD_CONV_STAGES=3 timeout -k 10 200 python bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/bench_resnet_s3.log 2>&1
echo "resnet s3 rc=$? $(tail -1 gpurun_out/bench_resnet_s3.log | cut -c1-200)"
exit 0
