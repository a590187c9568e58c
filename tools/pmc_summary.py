#!/usr/bin/env python3
"""Join rocprofv3 --pmc passes (p1, p2, ...) per dispatch and print per-kernel ratios.

    python tools/pmc_summary.py gpurun_out/pmc_conv [--filter conv_igemm]
    python tools/pmc_summary.py --gemm-check gpurun_out/pmcgemm/p1 struct.jsonl REPS

MFMA utilisation (round 5 normalisation, validated by --gemm-check on tools/probes/gemm_struct.hip):
every kernel here issues ``v_mfma_f32_16x16x32_bf16`` (16 x 16 x 32 x 2 = 16384 FLOP per wave
instruction). SQ_INSTS_MFMA counts MFMA wave-instructions over the whole chip, so

    MFMA util % = SQ_INSTS_MFMA x 16384 / (kernel duration x 2.5 PFLOP/s dense bf16)

— the fraction of the chip's dense bf16 peak the kernel's own MFMAs deliver over its own
duration, no clock assumption. SQ_VALU_MFMA_BUSY_CYCLES / SQ_INSTS_MFMA (the busy cycles counted
per MFMA) is printed as a check of the counter's units. Until round 4 the column divided the
busy cycles by GRBM_GUI_ACTIVE / 8 (the "effective clock"), which reads 2.5-5 GHz on dispatches
shorter than ~0.3 ms (MI355X_MICROARCH.md, DVFS give-back) and so under-stated every short
kernel; that column is gone.
"""
import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict

FLOP_PER_MFMA = 16 * 16 * 32 * 2
PEAK_FLOPS = 2.5e15


def load(root):
    disp = defaultdict(dict)
    names, dur = {}, {}
    for f in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
        pas = os.path.relpath(f, root).split(os.sep)[0]
        for r in csv.DictReader(open(f)):
            key = (pas, int(r["Dispatch_Id"]))
            disp[key][r["Counter_Name"]] = float(r["Counter_Value"])
            names[key] = r["Kernel_Name"]
            dur[key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
    merged = defaultdict(dict)
    for (p, d), v in disp.items():  # dispatch ids are identical across passes (same program)
        merged[d].update(v)
        merged[d]["_name"] = names[(p, d)]
        merged[d].setdefault("_us", dur[(p, d)])
    return merged


def util(v):
    return 100.0 * v.get("SQ_INSTS_MFMA", float("nan")) * FLOP_PER_MFMA / (v["_us"] * 1e-6 * PEAK_FLOPS)


def main(root, flt=""):
    merged = load(root)
    print("| id | us | kernel | MFMA util % of peak | busy cyc / MFMA | VALU/MFMA | LDS-conflict/LDS | "
          "wait-LDS % | wait-any % | L2 hit % | fabric read GB/s |")
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
        print(f"| {d} | {v['_us']:.1f} | `{n.split('(')[0][-48:]}` | {util(v):.1f} | "
              f"{g('SQ_VALU_MFMA_BUSY_CYCLES') / max(mf, 1):.1f} | "
              f"{g('SQ_INSTS_VALU') / max(mf, 1):.1f} | {g('SQ_LDS_BANK_CONFLICT') / max(g('SQ_INSTS_LDS'), 1):.2f} | "
              f"{100 * g('SQ_WAIT_INST_LDS') / max(wc, 1):.1f} | {100 * g('SQ_WAIT_ANY') / max(wc, 1):.1f} | "
              f"{100 * hit / max(hit + miss, 1):.1f} | "
              # FETCH_SIZE is in KB and reads 1/2 of a wide streaming read (MI355X_MICROARCH.md HBM)
              f"{2 * g('FETCH_SIZE') * 1024 / max(v['_us'], 1e-3) / 1e3:.0f} |")


def gemm_check(root, struct_path, reps):
    """Per gemm_struct configuration (3 warm-up + REPS launches of one kernel each): counted
    MFMA FLOP vs the GEMM's 2MNK, busy cycles per MFMA, counter-based vs time-based utilisation."""
    merged = load(root)
    cfgs = [json.loads(x) for x in open(struct_path) if x.strip().startswith("{")]
    ids = sorted(merged)
    per = 3 + reps
    if len(ids) != per * len(cfgs):
        print(f"warning: {len(ids)} dispatches for {len(cfgs)} configurations x {per}")
    print("| shape | tile | waves | counted MFMA FLOP / 2MNK | busy cyc / MFMA | util % (counters, kernel us) | "
          "util % (2MNK, kernel us) | util % (2MNK, event-timed loop) |")
    print("|---|---|---|---|---|---|---|---|")
    for i, c in enumerate(cfgs):
        ds = [merged[d] for d in ids[i * per + 3:(i + 1) * per]]
        if not ds:
            break
        flop = 2.0 * c["M"] * c["N"] * c["K"]
        ratio = statistics.median(v["SQ_INSTS_MFMA"] * FLOP_PER_MFMA / flop for v in ds)
        cyc = statistics.median(v["SQ_VALU_MFMA_BUSY_CYCLES"] / max(v["SQ_INSTS_MFMA"], 1) for v in ds)
        uc = statistics.median(util(v) for v in ds)
        ut = statistics.median(100.0 * flop / (v["_us"] * 1e-6 * PEAK_FLOPS) for v in ds)
        print(f"| {c['shape']} | {c['tile']} | {c['waves']} | {ratio:.3f} | {cyc:.1f} | {uc:.1f} | {ut:.1f} | "
              f"{100 * c['tflops'] / 2500:.1f} |")


if __name__ == "__main__":
    if sys.argv[1] == "--gemm-check":
        gemm_check(sys.argv[2], sys.argv[3], int(sys.argv[4]))
    else:
        main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
