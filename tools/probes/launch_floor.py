"""Per-dispatch cost floor on one MI355X: how long does a trivial kernel take back to back,
eagerly and replayed from a hipGraph, and how does it grow with the grid size?

    python tools/launch_floor.py [--n 200]

Prints one JSON line per case: us per dispatch = wall / n (events around the whole batch).
Used to decide how much a step gains from removing a launch (profiles/r2_launch_floor.md).
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=200)
    args = ap.parse_args()
    import torch
    import ddp_amd
    from ddp_amd.ops.common import native
    n = native()
    dev = torch.device("cuda", 0)
    buf = torch.zeros(1 << 24, dtype=torch.float32, device=dev)

    def run(kind, elems):
        s = torch.cuda.current_stream().cuda_stream
        for _ in range(args.n):
            if kind == "counter":
                n.counter_add(buf.data_ptr(), 1, s)
            else:
                n.scale(buf.data_ptr(), elems, 1.0, s)

    out = []
    for kind, elems in [("counter", 0), ("scale", 256), ("scale", 65536), ("scale", 1 << 20),
                        ("scale", 1 << 24)]:
        for mode in ("eager", "graph"):
            torch.cuda.synchronize()
            if mode == "graph":
                g = torch.cuda.CUDAGraph()
                st = torch.cuda.Stream()
                with torch.cuda.stream(st):
                    run(kind, elems)  # warm
                torch.cuda.synchronize()
                with torch.cuda.graph(g):
                    run(kind, elems)
                g.replay()
                torch.cuda.synchronize()
                fn = g.replay
            else:
                run(kind, elems)
                torch.cuda.synchronize()
                fn = lambda: run(kind, elems)  # noqa: E731
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            best = 1e9
            for _ in range(5):
                e0.record()
                fn()
                e1.record()
                e1.synchronize()
                best = min(best, e0.elapsed_time(e1) * 1000.0 / args.n)
            r = {"kernel": kind, "elems": elems, "mode": mode, "us_per_dispatch": round(best, 3),
                 "env": {k: v for k, v in os.environ.items() if k.startswith(("DEBUG_CLR", "HIP_", "GPU_"))}}
            out.append(r)
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
