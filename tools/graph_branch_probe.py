#!/usr/bin/env python3
"""Probe: cost of fork/join branches inside a captured hipGraph.

Captures 80 small kernels on one stream (linear graph) and the same 80 kernels with a side
branch forked/joined every `--every` kernels (the side branch runs one kernel), then times graph
replays. Prints one JSON line per variant. Used to decide how the step graph may use streams
(backward side stream, DDP comm stream) on this ROCm stack.
"""
import argparse
import json
import time

import torch


JOIN_END = False


def build(x, y, nk, every, side):
    main = torch.cuda.current_stream()
    for i in range(nk):
        x.mul_(1.0001)
        if side is not None and every and (i + 1) % every == 0:
            side.wait_stream(main)
            with torch.cuda.stream(side):
                y.add_(1.0)
            if not JOIN_END:
                main.wait_stream(side)
    if JOIN_END and every:
        main.wait_stream(side)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--every", type=int, default=10)
    ap.add_argument("--nk", type=int, default=80)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--priority", type=int, default=0, help="side stream priority (-1 = high)")
    ap.add_argument("--segmented", action="store_true")
    ap.add_argument("--nseg", type=int, default=8)
    ap.add_argument("--join-end", action="store_true", help="fork often, join once at the end")
    a = ap.parse_args()
    global JOIN_END
    JOIN_END = a.join_end
    if a.segmented:
        segmented(a.nk, a.nseg, a.iters)
        return
    dev = torch.device("cuda", 0)
    x = torch.ones(1 << 16, device=dev)
    y = torch.ones(1 << 10, device=dev)
    side = torch.cuda.Stream(priority=a.priority)
    out = {}
    for name, ev in (("linear", 0), ("branched", a.every)):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            build(x, y, a.nk, ev, side)  # warm-up
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            build(x, y, a.nk, ev, side)
        for _ in range(10):
            g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            g.replay()
        torch.cuda.synchronize()
        out[name] = (time.perf_counter() - t0) / a.iters * 1e6
        # eager reference
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            build(x, y, a.nk, ev, side)
        torch.cuda.synchronize()
        out[name + "_eager"] = (time.perf_counter() - t0) / 20 * 1e6
    print(json.dumps({k: round(v, 1) for k, v in out.items()}), flush=True)


def segmented(nk=80, nseg=8, iters=200):
    """The linear graph split into `nseg` captured segments; after each segment an eager side-
    stream kernel forks off (side waits on main), joined once at the end — the launch pattern of
    a step whose bucket collectives run eagerly on a comm stream between graph segments."""
    dev = torch.device("cuda", 0)
    x = torch.ones(1 << 16, device=dev)
    y = torch.ones(1 << 10, device=dev)
    side = torch.cuda.Stream()
    per = nk // nseg
    graphs = []
    pool = torch.cuda.graph_pool_handle()
    for _ in range(nseg):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(per):
                x.mul_(1.0001)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, pool=pool):
            for _ in range(per):
                x.mul_(1.0001)
        graphs.append(g)
    single = torch.cuda.CUDAGraph()
    with torch.cuda.graph(single, pool=pool):
        for _ in range(per * nseg):
            x.mul_(1.0001)
    main = torch.cuda.current_stream()
    res = {}
    for rep in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n = 10 if rep == 0 else iters
        for _ in range(n):
            single.replay()
        torch.cuda.synchronize()
        res["single"] = (time.perf_counter() - t0) / n * 1e6
    for mode in ("segments_only", "segments_side"):
        for rep in range(2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            n = 10 if rep == 0 else iters
            for _ in range(n):
                for g in graphs:
                    g.replay()
                    if mode == "segments_side":
                        side.wait_stream(main)
                        with torch.cuda.stream(side):
                            y.add_(1.0)
                if mode == "segments_side":
                    main.wait_stream(side)
            torch.cuda.synchronize()
            res[mode] = (time.perf_counter() - t0) / n * 1e6
    print(json.dumps({k: round(v, 1) for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
