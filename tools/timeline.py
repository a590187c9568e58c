"""Per-dispatch timeline of one training step from a rocprofv3 kernel trace.

    python tools/timeline.py gpurun_out/prof/vgg11 [step_index_from_end]
Prints start offset, duration, queue/stream and gap to the previous dispatch for the kernels
between two consecutive SGD launches (one captured step), to show stream overlap and idle gaps.
"""
import csv
import sys


def main(prefix, back="1"):
    trace = list(csv.DictReader(open(prefix + "_kernel_trace.csv")))
    trace.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(trace) if "sgd" in r["Kernel_Name"]]
    k = int(back)
    a, b = idx[-1 - k], idx[-k]
    step = trace[a + 1:b + 1]
    t0 = int(step[0]["Start_Timestamp"])
    qcol = next((c for c in ("Queue_Id", "Stream_Id", "Stream_Handle") if c in step[0]), None)
    print(f"columns: {list(step[0].keys())}")
    end = t0
    busy_end = t0
    idle = 0
    for r in step:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = s - busy_end
        if gap > 0:
            idle += gap
        busy_end = max(busy_end, e)
        q = r.get(qcol, "") if qcol else ""
        print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} q={q:>3} gap={gap / 1e3:7.1f}  {r['Kernel_Name'][:70]}")
        end = max(end, e)
    print(f"wall {(end - t0) / 1e3:.1f} us, idle (no kernel running) {idle / 1e3:.1f} us, "
          f"{len(step)} dispatches")


if __name__ == "__main__":
    main(*sys.argv[1:])
