#!/bin/bash
# round 5: det probe repeatability x3, then the GPU suite
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r5f; mkdir -p $O
for i in 1 2 3; do
  DDP_AMD_DETERMINISTIC=1 timeout -k 10 300 python tests/det_probe.py ddp > $O/det_ddp_$i.json 2> $O/det_ddp_$i.err || { tail -30 $O/det_ddp_$i.err; exit 1; }
  tail -1 $O/det_ddp_$i.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('diag', d['diag'], 'false', [k for k,v in d.items() if v is False and not k.endswith('/nan')])"
done
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { grep -E "FAIL|Error" $O/gpu_tests.log | head -20; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
