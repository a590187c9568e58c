#!/bin/bash
# round 5: deterministic-statistics build — bitwise execution comparisons
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r5e; mkdir -p $O
for c in ddp strategy divisor; do
  DDP_AMD_DETERMINISTIC=1 timeout -k 10 300 python tests/det_probe.py $c > $O/det_$c.json 2> $O/det_$c.err || { tail -30 $O/det_$c.err; exit 1; }
  cat $O/det_$c.json
done
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_deterministic.py tests/test_gpu_rccl_self.py > $O/tests.log 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.log | head -20; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
