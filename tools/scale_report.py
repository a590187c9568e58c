#!/usr/bin/env python3
"""Markdown table (images/s, ms/step, scaling efficiency vs 1 GPU) from tools/scale_sweep.sh.

    python tools/scale_report.py [gpurun_out/scale_sweep.jsonl]
Weak scaling efficiency = value(N) / (N * value(1)); strong = value(N) / (N * value(1)) too, as
throughput per GPU relative to one GPU running the same global batch.
"""
import json
import sys
from collections import defaultdict


def main(path="gpurun_out/scale_sweep.jsonl"):
    rows = [json.loads(l) for l in open(path) if l.strip()]
    by = defaultdict(dict)
    for r in rows:
        key = (r["config"]["strategy"], r["scaling"])
        by[key][r["n_gpus"]] = r
    print("| strategy | scaling | GPUs | images/s | ms/step | efficiency vs 1 GPU |")
    print("|---|---|---|---|---|---|")
    for (strat, scal), d in sorted(by.items()):
        base = d.get(1)
        for n in sorted(d):
            r = d[n]
            eff = (r["value"] / (n * base["value"])) if base else float("nan")
            print(f"| {strat} | {scal} | {n} | {r['value']:,.0f} | {r['ms_per_step']:.3f} | "
                  f"{eff * 100:.1f}% |")


if __name__ == "__main__":
    main(*sys.argv[1:])
