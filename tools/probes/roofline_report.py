#!/usr/bin/env python3
"""Markdown tables from tools/probes/roofline.py (--json) and gemm_struct.bin (JSON lines).

    python tools/probes/roofline_report.py --roofline gpurun_out/r4b/roofline.json \
        [--struct gpurun_out/r4c/gemm_struct.jsonl]
"""
import argparse
import json


def roofline_table(rows):
    out = ["| batch | layer | shape | GFLOP (fwd) | ours fwd us (TF/s) | hipBLASLt fwd us (TF/s) | "
           "ours bwd us (TF/s) | hipBLASLt dgrad+wgrad us (TF/s) | peak fwd / bwd us |",
           "|---|---|---|---|---|---|---|---|---|"]
    for r in rows:
        out.append(f"| {r['batch']} | {r['layer']} | {r['shape']} | {r['gflop_fwd']} | "
                   f"{r['ours_fwd_us']} ({r['ours_fwd_tflops']}) | {r['mm_fwd_us']} ({r['mm_fwd_tflops']}) | "
                   f"{r['ours_bwd_us']} ({r['ours_bwd_tflops']}) | "
                   f"{round(r['mm_dgrad_us'] + r['mm_wgrad_us'], 2)} ({r['mm_bwd_tflops']}) | "
                   f"{r['peak_fwd_us']} / {r['peak_bwd_us']} |")
    for b in sorted({r["batch"] for r in rows}):
        t = [r for r in rows if r["batch"] == b]
        of, mf = sum(r["ours_fwd_us"] for r in t), sum(r["mm_fwd_us"] for r in t)
        ob = sum(r["ours_bwd_us"] for r in t)
        mb = sum(r["mm_dgrad_us"] + r["mm_wgrad_us"] for r in t)
        out.append(f"| {b} | all | | | {of:.1f} | {mf:.1f} | {ob:.1f} | {mb:.1f} | |")
    return "\n".join(out)


def struct_table(lines):
    rows = [json.loads(x) for x in lines if x.strip().startswith("{")]
    out = ["| shape | M x N x K (splits) | tile | waves | ring | k-steps/barrier | LDS KB | blocks | us | TF/s | max rel err |",
           "|---|---|---|---|---|---|---|---|---|---|---|"]
    best = {}
    for r in rows:
        out.append(f"| {r['shape']} | {r['M']} x {r['N']} x {r['K']} ({r['splits']}) | {r['tile']} | "
                   f"{r['waves']} | {r['nst']} | {r['kpb']} | {r['lds_kb']} | {r['blocks']} | "
                   f"{r['us']:.2f} | {r['tflops']:.0f} | {r['max_rel_err']:.1e} |")
        if r["shape"] not in best or r["us"] < best[r["shape"]]["us"]:
            best[r["shape"]] = r
    out.append("")
    out.append("Best per shape: " + ", ".join(
        f"{k} {v['tile']}/{v['waves']}/nst{v['nst']}/kpb{v['kpb']} {v['us']:.1f} us ({v['tflops']:.0f} TF/s)"
        for k, v in best.items()))
    return "\n".join(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--roofline")
    ap.add_argument("--struct")
    a = ap.parse_args()
    if a.roofline:
        print(roofline_table(json.load(open(a.roofline))))
        print()
    if a.struct:
        print(struct_table(open(a.struct).read().splitlines()))


if __name__ == "__main__":
    main()
