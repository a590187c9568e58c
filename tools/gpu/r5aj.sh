#!/bin/bash
# round 5: BN kernel tests + kernel-level profile of the current tree (VGG-11 b256) after
# restoring the reduce / forward-apply load order; + 3 interleaved bench pairs vs _oldtree/
cd "$GRAFT_REPO_ROOT" || exit 2
O=$GRAFT_REPO_ROOT/gpurun_out/r5aj; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_resnet.py -k "bn_act or resnet" -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAIL|Error" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
mkdir -p gpurun_out/prof
P=$GRAFT_REPO_ROOT/gpurun_out/prof/r5aj_new
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$P" -o p -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 --ref-window 0 > "$P.log" 2>&1) || { tail -5 "$P.log"; exit 1; }
for i in 1 2 3; do
  for t in new old; do
    if [ $t = old ]; then D=$GRAFT_REPO_ROOT/_oldtree; else D=$GRAFT_REPO_ROOT; fi
    (cd $D && timeout -k 10 200 python bench.py --steps 60 --warmup 10 > $O/b256_${t}_$i.log 2>&1) || { tail -5 $O/b256_${t}_$i.log; exit 1; }
    tail -1 $O/b256_${t}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('b256 $t', d['ms_per_step'], d['value'])"
  done
done
