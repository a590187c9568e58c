"""Summarise a rocprofv3 --kernel-trace --stats run (CSV) into markdown.

    python tools/prof_summary.py gpurun_out/prof/vgg11 [title] > profiles/xyz.md
Reads <prefix>_kernel_stats.csv and <prefix>_kernel_trace.csv; prints the top kernels and one
training step (the dispatches between the last two SGD kernels) in launch order.
"""
import csv
import sys


def main(prefix, title="rocprofv3 kernel summary"):
    stats = list(csv.DictReader(open(prefix + "_kernel_stats.csv")))
    # (rocprofv3 writes the rows in completion / buffer order, not launch order)
    trace = sorted(csv.DictReader(open(prefix + "_kernel_trace.csv")),
                   key=lambda r: int(r["Start_Timestamp"]))
    print(f"# {title}\n")
    print("## Top kernels (whole run)\n")
    print("| kernel | calls | total ms | avg us | % |")
    print("|---|---|---|---|---|")
    for r in sorted(stats, key=lambda r: -float(r["TotalDurationNs"]))[:20]:
        print(f"| `{r['Name'][:90]}` | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.3f} | "
              f"{float(r['AverageNs']) / 1e3:.1f} | {float(r['Percentage']):.1f} |")
    idx = [i for i, r in enumerate(trace) if "sgd" in r["Kernel_Name"]]
    if len(idx) >= 2:
        a, b = idx[-2], idx[-1]
        step = trace[a + 1:b + 1]
        t0 = int(step[0]["Start_Timestamp"])
        t1 = int(step[-1]["End_Timestamp"])
        busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in step)
        print(f"\n## One training step ({len(step)} dispatches, wall {(t1 - t0) / 1e3:.1f} us, "
              f"kernel-busy {busy / 1e3:.1f} us)\n")
        print("| us | grid (WGs) | VGPR | LDS | kernel |")
        print("|---|---|---|---|---|")
        for r in step:
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            wg = int(r["Workgroup_Size_X"]) or 1
            g = f"{int(r['Grid_Size_X']) // wg}x{r['Grid_Size_Y']}x{r['Grid_Size_Z']}"
            print(f"| {d:.1f} | {g} | {r.get('VGPR_Count', '')} | {r.get('LDS_Block_Size', '')} | "
                  f"`{r['Kernel_Name'][:80]}` |")


if __name__ == "__main__":
    main(*sys.argv[1:])
