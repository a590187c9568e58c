#!/usr/bin/env python3
"""Join rocprofv3 --pmc passes (p1, p2, ...) per dispatch and print per-kernel ratios.

    python tools/pmc_summary.py gpurun_out/pmc_conv [--filter conv_igemm]
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(root, flt=""):
    disp = defaultdict(dict)
    names, dur = {}, {}
    for f in sorted(glob.glob(os.path.join(root, "p*", "*counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            key = (os.path.basename(os.path.dirname(f)), int(r["Dispatch_Id"]))
            disp[key][r["Counter_Name"]] = float(r["Counter_Value"])
            names[key] = r["Kernel_Name"]
            dur[key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
    # dispatch ids are identical across passes (same program): merge by id
    merged = defaultdict(dict)
    for (p, d), v in disp.items():
        merged[d].update(v)
        merged[d]["_name"] = names[(p, d)]
        merged[d].setdefault("_us", dur[(p, d)])
    print("| id | us | kernel | MFMA busy/wave-cyc | VALU/MFMA | LDS-conflict/LDS | wait-LDS % | wait-any % | L2 hit % |")
    print("|---|---|---|---|---|---|---|---|---|")
    for d in sorted(merged):
        v = merged[d]
        n = v["_name"]
        if flt and flt not in n:
            continue
        g = lambda k: v.get(k, float("nan"))  # noqa: E731
        wc = g("SQ_WAVE_CYCLES")
        mf = g("SQ_INSTS_MFMA")
        hit, miss = g("TCC_HIT_sum"), g("TCC_MISS_sum")
        print(f"| {d} | {v['_us']:.1f} | `{n.split('(')[0][-48:]}` | "
              f"{g('SQ_VALU_MFMA_BUSY_CYCLES') / max(g('SQ_BUSY_CYCLES'), 1):.2f} | "
              f"{g('SQ_INSTS_VALU') / max(mf, 1):.1f} | {g('SQ_LDS_BANK_CONFLICT') / max(g('SQ_INSTS_LDS'), 1):.2f} | "
              f"{100 * g('SQ_WAIT_INST_LDS') / max(wc, 1):.1f} | {100 * g('SQ_WAIT_ANY') / max(wc, 1):.1f} | "
              f"{100 * hit / max(hit + miss, 1):.1f} |")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
