"""How much of each collective kernel's time ran concurrently with compute kernels
(rocprofv3 kernel trace CSV). Collective = kernel name containing 'nccl', 'rccl' or 'oneRank' (RCCL's
device kernels); compute = everything else except the 1-wave flag waits.

    python tools/overlap_report.py OUT/ovl_kernel_trace.csv [--last N]
"""
import csv
import sys


def main(path, last=None):
    rows = list(csv.DictReader(open(path)))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
    ks.sort()
    coll = [k for k in ks if any(t in k[2].lower() for t in ("nccl", "rccl", "onerank"))]
    comp = [k for k in ks if k not in coll and "flag_wait" not in k[2]]
    if last:
        coll = coll[-int(last):]
    print(f"{len(coll)} collective kernels, {len(comp)} compute kernels")
    print("| collective | dur us | overlapped us | % | concurrent compute kernels |")
    print("|---|---|---|---|---|")
    tot_d = tot_o = 0
    for s, e, n in coll:
        ov, names = 0, set()
        for cs, ce, cn in comp:
            lo, hi = max(s, cs), min(e, ce)
            if hi > lo:
                ov += hi - lo
                names.add(cn.split("(")[0].replace("void ", "").replace("ddp_amd::", "")[:40])
        ov = min(ov, e - s)
        tot_d += e - s
        tot_o += ov
        print(f"| `{n[:50]}` | {(e - s) / 1e3:.1f} | {ov / 1e3:.1f} | {100 * ov / max(e - s, 1):.0f} | "
              f"{', '.join(sorted(names)[:4])} |")
    if tot_d:
        print(f"\ntotal: {tot_d / 1e3:.1f} us of collectives, {tot_o / 1e3:.1f} us "
              f"({100 * tot_o / tot_d:.0f}%) concurrent with compute")


if __name__ == "__main__":
    main(*sys.argv[1:])
