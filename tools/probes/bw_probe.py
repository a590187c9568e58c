#!/usr/bin/env python3
"""HBM bandwidth ceilings for the activation sizes of ResNet-50 b256 (411 MB bf16): write-only
(fill), read-only (sum), copy."""
import torch

def t(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / reps

for mb in (103, 411):
    n = mb * 1000 * 1000 // 2 // 1024 * 1024
    x = torch.empty(n, dtype=torch.bfloat16, device="cuda")
    y = torch.empty_like(x)
    x.fill_(1)
    us = t(lambda: y.fill_(0))
    print(f"{mb} MB fill  {us:7.1f} us {mb / us:5.2f} TB/s")
    us = t(lambda: y.copy_(x))
    print(f"{mb} MB copy  {us:7.1f} us {2 * mb / us:5.2f} TB/s (r+w)")
    xf = x.view(-1, 1024)
    us = t(lambda: xf.sum(dim=0))
    print(f"{mb} MB sum   {us:7.1f} us {mb / us:5.2f} TB/s")
