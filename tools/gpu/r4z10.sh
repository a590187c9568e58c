#!/bin/bash
# round 4: re-tune the b128 / b256 backward-pair entries, then whole-step A/B of each changed entry
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r4z10; mkdir -p $O
TABLE=distributed-data-parallel-ml-training_amd/ops/conv_tuning.json
cp $TABLE $O/base.json
timeout -k 10 600 python -u tools/conv_tune.py --pairs --pair-sets vgg11:128,256 --reps 40 \
    --merge $O/base.json --out $O/new.json > $O/tune.log 2>&1 || { tail -20 $O/tune.log; exit 1; }
grep -v amdgpu.ids $O/tune.log
python3 - <<'PY'
import json
O = "gpurun_out/r4z10"
key = lambda e: (e["mode"], e["M"], e["N"], e["K"])
base = json.load(open(f"{O}/base.json")); new = json.load(open(f"{O}/new.json"))
bm = {key(e): e for e in base["entries"]}
n = 0
for e in new["entries"]:
    if e["mode"] != 3:
        continue
    o = bm.get(key(e))
    if o is not None and (o["tile"], o["splits"], o["stages"]) == (e["tile"], e["splits"], e["stages"]):
        continue
    t = json.load(open(f"{O}/base.json"))
    t["entries"] = [x for x in t["entries"] if key(x) != key(e)] + [e]
    json.dump(t, open(f"{O}/v{n}.json", "w"), indent=1)
    B = int(e["shape"].split()[1][1:])
    open(f"{O}/v{n}.batch", "w").write(str(B))
    print(f"v{n}", e["shape"], e["tile"], e["splits"], e["stages"], "base", (o["tile"], o["splits"], o["stages"]) if o else None)
    n += 1
PY
for P in 1 2; do
  for f in $O/v*.json; do
    T=$(basename $f .json); B=$(cat $O/$T.batch)
    for X in base $T; do
      cp $O/$X.json $TABLE
      L=$O/b${B}_${X}_${T}_p$P.log
      timeout -k 10 200 python bench.py --global-batch $B --steps 60 --warmup 10 --ref-window 0 > $L 2>&1 || { tail -5 $L; cp $O/base.json $TABLE; exit 1; }
      echo "b$B $X (vs $T) p$P $(tail -1 $L | grep -oE '"ms_per_step": [0-9.]+')"
    done
  done
done
cp $O/base.json $TABLE
