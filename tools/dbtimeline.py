"""Per-dispatch timeline of one training step from a rocprofv3 rocpd database (ROCm 7 default
output): python tools/dbtimeline.py gpurun_out/prof_seg/seg4dev_results.db [steps_back]
Prints start offset, duration, gap to the previous busy end, queue/stream, kernel name for the
dispatches between two consecutive SGD launches; gaps > 2 us are summed."""
import sqlite3
import sys


def main(db, back="2"):
    c = sqlite3.connect(db)
    rows = list(c.execute("select name,start,end,queue_id,stream_id from kernels order by start"))
    idx = [i for i, r in enumerate(rows) if "sgd" in r[0]]
    k = int(back)
    a, b = idx[-1 - k], idx[-k]
    step = rows[a + 1:b + 1]
    t0 = rows[a][2]
    busy, gaps = t0, 0.0
    for r in step:
        gap = (r[1] - busy) / 1e3
        if gap > 2:
            gaps += gap
        print(f"{(r[1] - t0) / 1e3:8.1f} {(r[2] - r[1]) / 1e3:6.1f} gap {gap:7.1f} q{r[3]} s{r[4]} {r[0][:60]}")
        busy = max(busy, r[2])
    print(f"step wall {(step[-1][2] - t0) / 1e3:.1f} us, idle gaps > 2 us: {gaps:.1f} us")


if __name__ == "__main__":
    main(*sys.argv[1:])
