"""All-reduce bandwidth sweep over a communicator ("measure ncclAllReduce bus
bandwidth versus size before fixing bucket sizes").

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 tools/comm_bench.py [--dtype bf16]

Per message size: mean time of ``iters`` back-to-back all-reduces (after ``warmup``), the
algorithm bandwidth bytes / t and the ring bus bandwidth algbw * 2 (n - 1) / n (nccl-tests
convention), max over ranks. Works with the native RCCL communicator (GPU, timed with
synchronize) and the Gloo TorchCommunicator (CPU tests). Also checks the result of the first
call (every rank contributes rank + 1, so each element must equal n (n + 1) / 2).
"""
import time

import torch
import torch.distributed as dist

from .comm import SUM


def default_sizes(lo=1 << 16, hi=1 << 27):
    s, out = lo, []
    while s <= hi:
        out.append(s)
        s *= 4
    return out


def allreduce_sweep(comm, sizes, dtype=torch.float32, device="cpu", iters=20, warmup=5):
    is_cuda = torch.device(device).type == "cuda"
    esize = torch.tensor([], dtype=dtype).element_size()
    n = comm.world
    rows = []

    def sync():
        if is_cuda:
            torch.cuda.synchronize()

    for nbytes in sizes:
        numel = max(1, nbytes // esize)
        t = torch.full((numel,), float(comm.rank + 1), dtype=dtype, device=device)
        comm.all_reduce(t, SUM)
        sync()
        ok = bool((t.float() == n * (n + 1) / 2).all().item()) if n > 1 else True
        for _ in range(warmup):
            comm.all_reduce(t, SUM)
        sync()
        if dist.is_initialized() and n > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(iters):
            comm.all_reduce(t, SUM)
        sync()
        dt = (time.perf_counter() - t0) / iters
        if dist.is_initialized() and n > 1:
            m = torch.tensor([dt], dtype=torch.float64)
            dist.all_reduce(m, op=dist.ReduceOp.MAX)
            dt = float(m.item())
        algbw = numel * esize / dt / 1e9
        rows.append({"bytes": numel * esize, "us": round(dt * 1e6, 2), "algbw_GBps": round(algbw, 3),
                     "busbw_GBps": round(algbw * 2 * (n - 1) / n, 3) if n > 1 else None,
                     "correct": ok})
    return rows


def shard_sweep(comm, sizes, device="cpu", iters=20, warmup=5):
    """Per fp32 bucket size S: mean time of a reduce-scatter(avg) of S bytes of fp32 and of an
    all-gather of S/2 bytes of bf16 (the sharded update's two collectives, parallel/zero.py
    ShardedBf16Update), max over ranks -> ``{"bytes", "rs_us", "ag16_us"}`` rows (merged into the
    all-reduce rows by bucket_plan.probe_table; priced by parallel/cut_plan.py shard16_us)."""
    from .comm import AVG
    is_cuda = torch.device(device).type == "cuda"
    n = comm.world
    rows = []

    def sync():
        if is_cuda:
            torch.cuda.synchronize()

    def timed(fn):
        for _ in range(warmup):
            fn()
        sync()
        if dist.is_initialized() and n > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        sync()
        dt = (time.perf_counter() - t0) / iters
        if dist.is_initialized() and n > 1:
            m = torch.tensor([dt], dtype=torch.float64)
            dist.all_reduce(m, op=dist.ReduceOp.MAX)
            dt = float(m.item())
        return round(dt * 1e6, 2)

    for nbytes in sizes:
        numel = max(n * 4, nbytes // 4 // (4 * n) * (4 * n))
        g = torch.ones(numel, dtype=torch.float32, device=device)
        w = torch.zeros(numel, dtype=torch.bfloat16, device=device)
        wv = w if is_cuda else w.view(torch.int32)  # Gloo: bf16 pairs as int32 words
        rs = timed(lambda: comm.reduce_scatter_inplace(g, AVG))
        ag = timed(lambda: comm.all_gather_inplace(wv))
        rows.append({"bytes": numel * 4, "rs_us": rs, "ag16_us": ag})
    return rows
