#!/bin/bash
# round 5: ResNet stem BN + 3x3 pool passes — grid caps (DDP_AMD_POOL3_GRIDS=fwd,reduce,apply)
# timed from kernel traces of short ResNet-50 b256 runs
cd "$GRAFT_REPO_ROOT" || exit 2
O=$GRAFT_REPO_ROOT/gpurun_out/r5az; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "maxpool3" -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
i=0
for cfg in ${CFGS:-8192,4096,16384 25088,4096,16384 16384,8192,25088 4096,2048,8192 25088,16384,50176}; do
  i=$((i+1))
  (cd /tmp && export TMPDIR=/tmp && DDP_AMD_POOL3_GRIDS=$cfg timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/p$i" -o p -- python3 "$GRAFT_REPO_ROOT/bench.py" --model resnet50 --steps 4 --warmup 2 --ref-window 0 > "$O/p$i.log" 2>&1) || { tail -5 "$O/p$i.log"; exit 1; }
  F=$(ls $O/p$i/*/p_kernel_stats.csv $O/p$i/p_kernel_stats.csv 2>/dev/null | head -1)
  python3 - "$F" "$cfg" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
out = []
for r in rows:
    n = r["Name"]
    if "pool3" in n:
        out.append(f"{n.split('(')[0].split()[-1]}={float(r['AverageNs'])/1000:.1f}us")
print(sys.argv[2], " ".join(sorted(out)))
PY
done
