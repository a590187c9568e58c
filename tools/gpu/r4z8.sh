#!/bin/bash
# round 4: confirm the b32 pair-table entry (16x16 layer, DGRAD split 2 / WGRAD 16) vs the old one
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r4z8; mkdir -p $O
TABLE=distributed-data-parallel-ml-training_amd/ops/conv_tuning.json
cp $TABLE $O/new.json
git_old=$O/old.json
python3 - <<'PY'
import json
t = json.load(open("gpurun_out/r4z8/new.json"))
for e in t["entries"]:
    if e["mode"] == 3 and e.get("shape", "").startswith("vgg11 N32 64->128 16x16"):
        e.update({"splits": 1, "stages": 8})
json.dump(t, open("gpurun_out/r4z8/old.json", "w"), indent=1)
PY
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for P in 1 2 3; do for T in old new; do
  cp $O/$T.json $TABLE
  L=$O/b32_${T}_p$P.log
  timeout -k 10 200 python bench.py --global-batch 32 --steps 60 --warmup 10 --ref-window 0 > $L 2>&1 || { tail -5 $L; cp $O/new.json $TABLE; exit 1; }
  echo "b32 $T p$P $(tail -1 $L | grep -oE '"ms_per_step": [0-9.]+')"
done; done
cp $O/new.json $TABLE
