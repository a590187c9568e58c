#!/bin/bash
# round 5: pair kernel with the master-SGD epilogue as a template switch (SGDM) — SGD / model /
# kernel tests, kernel profile at b256, b32 / b256 benches
cd "$GRAFT_REPO_ROOT" || exit 2
O=$GRAFT_REPO_ROOT/gpurun_out/r5ak; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_deterministic.py tests/test_gpu_kernels.py -k "sgd or pair or deterministic or oracle or conv" -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAIL|Error" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
mkdir -p gpurun_out/prof
P=$GRAFT_REPO_ROOT/gpurun_out/prof/r5ak_new
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$P" -o p -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 --ref-window 0 > "$P.log" 2>&1) || { tail -5 "$P.log"; exit 1; }
for b in 256 32; do
  for i in 1 2; do
    timeout -k 10 200 python bench.py --global-batch $b --steps 60 --warmup 10 > $O/b${b}_$i.log 2>&1 || { tail -5 $O/b${b}_$i.log; exit 1; }
    tail -1 $O/b${b}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('b$b', d['ms_per_step'], d['value'])"
  done
done
