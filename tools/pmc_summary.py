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
    for f in sorted(glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            key = (os.path.relpath(f, root).split(os.sep)[0], int(r["Dispatch_Id"]))
            disp[key][r["Counter_Name"]] = float(r["Counter_Value"])
            names[key] = r["Kernel_Name"]
            dur[key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
    # dispatch ids are identical across passes (same program): merge by id
    merged = defaultdict(dict)
    for (p, d), v in disp.items():
        merged[d].update(v)
        merged[d]["_name"] = names[(p, d)]
        merged[d].setdefault("_us", dur[(p, d)])
    # MFMA util = MFMA-busy cycles / (effective clock cycles x 1024 SIMDs); effective clock =
    # GRBM_GUI_ACTIVE / 8 XCDs / wall (MI355X_MICROARCH.md 'DVFS give-back'; reads high < 0.3 ms)
    print("| id | us | kernel | MFMA util % | clk GHz | VALU/MFMA | LDS-conflict/LDS | wait-LDS % | wait-any % | L2 hit % | fabric read GB/s |")
    print("|---|---|---|---|---|---|---|---|---|---|---|")
    for d in sorted(merged):
        v = merged[d]
        n = v["_name"]
        if flt and flt not in n:
            continue
        g = lambda k: v.get(k, float("nan"))  # noqa: E731
        wc = g("SQ_WAVE_CYCLES")
        mf = g("SQ_INSTS_MFMA")
        hit, miss = g("TCC_HIT_sum"), g("TCC_MISS_sum")
        cyc = g("GRBM_GUI_ACTIVE") / 8.0
        print(f"| {d} | {v['_us']:.1f} | `{n.split('(')[0][-48:]}` | "
              f"{100 * g('SQ_VALU_MFMA_BUSY_CYCLES') / max(cyc * 1024, 1):.1f} | "
              f"{cyc / max(v['_us'], 1e-3) / 1000:.2f} | "
              f"{g('SQ_INSTS_VALU') / max(mf, 1):.1f} | {g('SQ_LDS_BANK_CONFLICT') / max(g('SQ_INSTS_LDS'), 1):.2f} | "
              f"{100 * g('SQ_WAIT_INST_LDS') / max(wc, 1):.1f} | {100 * g('SQ_WAIT_ANY') / max(wc, 1):.1f} | "
              f"{100 * hit / max(hit + miss, 1):.1f} | "
              # FETCH_SIZE is in KB and reads 1/2 of a wide streaming read (MI355X_MICROARCH.md HBM)
              f"{2 * g('FETCH_SIZE') * 1024 / max(v['_us'], 1e-3) / 1e3:.0f} |")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
