#!/usr/bin/env python3
"""Do the parallel branches of ONE captured hipGraph run concurrently on this ROCm?
Two spin kernels (torch.cuda._sleep) on forked streams inside one capture vs back to back."""
import torch

def timed(g, reps=20):
    g.replay(); torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        g.replay()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / reps

CYC = 200000
main = torch.cuda.Stream()
side = torch.cuda.Stream()
side_hi = torch.cuda.Stream(priority=-1)
res = {}
for name in ("serial", "branches", "branches_hiprio"):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(main):
        torch.cuda._sleep(CYC)
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=main):
            if name == "serial":
                torch.cuda._sleep(CYC)
                torch.cuda._sleep(CYC)
            else:
                s = side if name == "branches" else side_hi
                s.wait_stream(main)
                with torch.cuda.stream(s):
                    torch.cuda._sleep(CYC)
                torch.cuda._sleep(CYC)
                main.wait_stream(s)
    res[name] = timed(g)
g1 = torch.cuda.CUDAGraph()
with torch.cuda.stream(main):
    with torch.cuda.graph(g1, stream=main):
        torch.cuda._sleep(CYC)
res["single"] = timed(g1)
print({k: round(v, 1) for k, v in res.items()})
