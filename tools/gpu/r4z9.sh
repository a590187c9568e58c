#!/bin/bash
# round 4: b64 pair-table entries one at a time (whole-step A/B of each re-tuned entry)
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r4z9; mkdir -p $O
TABLE=distributed-data-parallel-ml-training_amd/ops/conv_tuning.json
cp $TABLE $O/base.json
NV=$(python3 -c "import json; print(len(json.load(open('tools/gpu/r4z9_variants.json'))))")
for i in $(seq 0 $((NV-1))); do
python3 - $i <<'PY'
import json, sys
i = int(sys.argv[1])
v = json.load(open("tools/gpu/r4z9_variants.json"))[i]
t = json.load(open("gpurun_out/r4z9/base.json"))
key = lambda e: (e["mode"], e["M"], e["N"], e["K"])
t["entries"] = [e for e in t["entries"] if key(e) != key(v)] + [v]
json.dump(t, open(f"gpurun_out/r4z9/v{i}.json", "w"), indent=1)
print(i, v["shape"], v["tile"], v["splits"], v["stages"])
PY
done
for P in 1 2; do for T in base $(seq -f "v%g" 0 $((NV-1))); do
  cp $O/$T.json $TABLE
  L=$O/b64_${T}_p$P.log
  timeout -k 10 200 python bench.py --global-batch 64 --steps 60 --warmup 10 --ref-window 0 > $L 2>&1 || { tail -5 $L; cp $O/base.json $TABLE; exit 1; }
  echo "b64 $T p$P $(tail -1 $L | grep -oE '"ms_per_step": [0-9.]+')"
done; done
cp $O/base.json $TABLE
