#!/usr/bin/env python3
"""Kernel-duration roofline: per-phase sums of a rocprofv3 kernel trace of
``tools/probes/roofline.py --trace phases.json`` (marker kernels' grid sizes give the phase ids).

    python tools/probes/roofline_trace.py phases.json <prefix>_kernel_trace.csv > table.md

Per layer and GEMM: ours (our kernels as trained, incl. BN statistics / split-K finish) and
hipBLASLt (torch.matmul of the same M x N x K, materialised operands) as the SUM OF KERNEL
DURATIONS per call (no launch gaps), TF/s, and the fraction of the 2.5 PF dense bf16 peak."""
import csv
import json
import sys
from collections import defaultdict

PEAK = 2500.0


def main(phases_path, trace_path):
    meta = json.load(open(phases_path))
    phases = {p["id"]: p for p in meta["phases"]}
    rows = sorted(csv.DictReader(open(trace_path)), key=lambda r: int(r["Start_Timestamp"]))
    cur, tot, names = None, defaultdict(float), defaultdict(set)
    for r in rows:
        n = r["Kernel_Name"]
        if "fill_bytes_kernel" in n:
            wg = int(r["Grid_Size_X"]) // max(int(r["Workgroup_Size_X"]), 1)
            cur = wg - 1 if wg - 1 in phases else None
            continue
        if cur:
            tot[cur] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
            names[cur].add(n.split("(")[0][-40:])
    per = {}
    for pid, p in phases.items():
        B, li, what = p["label"]
        per[(B, li, what)] = tot[pid] / p["reps"]
    out = ["| batch | layer | shape | GFLOP fwd | ours fwd us (TF/s, % peak) | hipBLASLt fwd us (TF/s) | "
           "ours bwd us (TF/s, % peak) | hipBLASLt dgrad + wgrad us (TF/s) |", "|---|---|---|---|---|---|---|---|"]
    sums = defaultdict(lambda: defaultdict(float))
    for r in meta["rows"]:
        B, li, gf = r["batch"], r["layer"], r["gflop_fwd"]
        of, mf = per[(B, li, "ours_fwd")], per[(B, li, "mm_fwd")]
        ob = per[(B, li, "ours_bwd")]
        bgf = gf if li == 0 else 2 * gf
        mb = per[(B, li, "mm_wgrad")] + (0 if li == 0 else per[(B, li, "mm_dgrad")])
        for k, v in (("of", of), ("mf", mf), ("ob", ob), ("mb", mb)):
            sums[B][k] += v
        tf = lambda g, us: g / us * 1e3 if us > 0 else 0.0  # noqa: E731
        out.append(f"| {B} | {li} | {r['shape']} | {gf} | {of:.2f} ({tf(gf, of):.0f}, {100 * tf(gf, of) / PEAK:.0f} %) | "
                   f"{mf:.2f} ({tf(gf, mf):.0f}) | {ob:.2f} ({tf(bgf, ob):.0f}, {100 * tf(bgf, ob) / PEAK:.0f} %) | "
                   f"{mb:.2f} ({tf(bgf, mb):.0f}) |")
    for B, s in sorted(sums.items()):
        out.append(f"| {B} | all | | | {s['of']:.1f} | {s['mf']:.1f} | {s['ob']:.1f} | {s['mb']:.1f} |")
    print("\n".join(out))
    print()
    print("Kernels per phase: " + "; ".join(f"{phases[k]['label']}: {sorted(v)}" for k, v in
                                           sorted(names.items())[:6]) + " ...")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
