#!/bin/bash
# round 4: full GPU suite + smoke + default bench + ResNet-50 on the shipped build
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r4p; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { grep -E "FAIL|Error" $O/gpu_tests.log | head -20; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 200 python bench.py > $O/bench_default.log 2>&1 || { tail -5 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log
timeout -k 10 300 python bench.py --model resnet50 --steps 8 --warmup 4 --ref-window 0 > $O/resnet.log 2>&1 || { tail -5 $O/resnet.log; exit 1; }
tail -1 $O/resnet.log | cut -c1-200
