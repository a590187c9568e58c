#!/usr/bin/env python3
"""Per-call cost of the BatchNorm kernels in a captured chain (no other kernels around them),
to compare with their cost inside the training step's kernel sequence."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import ddp_amd  # noqa: F401
from ddp_amd.ops.common import native, ptr, stream_handle

nat = native()
DEV = "cuda"
REPS = 100


def chain(fn, reps=REPS):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                fn()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(5):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / (5 * reps)


for (N, C, H, pool) in [(32, 128, 16, True), (32, 256, 8, False), (32, 512, 4, True),
                        (32, 512, 2, False), (256, 256, 8, False)]:
    zn = torch.randn(N, H, H, C, device=DEV).to(torch.bfloat16)
    stats = torch.rand(16, 2 * C, device=DEV)
    gamma = torch.rand(C, device=DEV) + 0.5
    beta = torch.randn(C, device=DEV) * 0.1
    Ho = H // 2 if pool else H
    out = torch.empty(N, Ho, Ho, C, device=DEV, dtype=torch.bfloat16)
    coef = torch.empty(6 * C, device=DEV)
    doutn = torch.randn(N, Ho, Ho, C, device=DEV).to(torch.bfloat16)
    sums = torch.zeros(16 * 2 * C, device=DEV)
    dz = torch.empty_like(zn)
    dg = torch.zeros(C, device=DEV)
    db = torch.zeros(C, device=DEV)

    def fwd():
        nat.bn_act_fwd(N, H, H, C, int(pool), 1, 1e-5, ptr(zn), 0, ptr(stats), ptr(gamma),
                       ptr(beta), ptr(out), stream_handle(), coef=ptr(coef))

    def bwd():
        nat.bn_act_bwd(N, H, H, C, int(pool), 1, 1e-5, ptr(zn), 0, ptr(stats), ptr(gamma),
                       ptr(beta), ptr(doutn), ptr(sums), ptr(dz), 0, ptr(dg), ptr(db), 0,
                       stream_handle(), ptr(coef), 0)
    print(f"N{N} C{C} {H}x{H} pool={int(pool)}: fwd {chain(fwd):5.2f} us/call, "
          f"bwd (reduce+finalize+apply) {chain(bwd):5.2f} us/call", flush=True)
