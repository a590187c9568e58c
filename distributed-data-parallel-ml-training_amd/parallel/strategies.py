"""Per-parameter gradient synchronisation strategies (run after the whole backward).

2A — centralised gather -> mean -> scatter (reference: part2/part2a/main.py:97-115).
     For each parameter in ``model.parameters()`` order rank 0 gathers every rank's gradient,
     averages them, and scatters the mean back. On RCCL the gather is a grouped ncclRecv from
     every peer into a [world, n] staging buffer (each peer on its own xGMI link), the mean is
     the ``mean_ws`` HIP kernel, and the scatter is a grouped ncclSend of the same buffer.
2B — per-parameter all-reduce(SUM) then ``grad /= world`` (reference: part2/part2b/main.py:97-103).
     On RCCL: ncclAllReduce(sum) + the ``scale`` HIP kernel, both on the compute stream.

Both are deliberately serial and blocking per parameter, like the reference (no bucketing, no
overlap) — that is what part 3 (parallel/ddp.py) improves on.
"""
import torch

from .comm import SUM, is_live


def _params_with_grad(model):
    return [p for p in model.parameters() if p.grad is not None]


def sync_gradients_gather_scatter(model, comm, root=0):
    """2A: rank-0 gather, mean, scatter of ``[mean] * world`` for every parameter."""
    if not is_live(comm):
        return  # the mean over one replica is the gradient itself
    params = _params_with_grad(model)
    if comm.kind == "torch":
        for p in params:
            lst = comm.gather(p.grad, dst=root)
            if comm.rank == root:
                p.grad.copy_(torch.mean(torch.stack(lst), dim=0))
            comm.scatter_replicated(p.grad, src=root)
        return
    from ..ops.common import native, stream_handle
    maxn = max(p.grad.numel() for p in params)
    staging = None
    if comm.rank == root:
        staging = _staging(params[0].grad.device, comm.world, maxn)
    if comm.world == 1 and hasattr(comm, "reserve_staging"):
        # single-rank RCCL: the self send/recv of the scatter lands in a staging buffer that
        # must exist before a capture (no allocation inside a captured step)
        comm.reserve_staging(maxn * params[0].grad.element_size())
    s = stream_handle()
    for p in params:
        g = p.grad
        n = g.numel()
        buf = staging[:comm.world * n].view(comm.world, n) if staging is not None else None
        comm.gather_into(g, buf, dst=root)
        if comm.rank == root:
            native().mean_ws(buf.data_ptr(), n, comm.world, g.data_ptr(), s)
        comm.scatter_replicated(g, src=root)


def sync_gradients_gather_broadcast(model, comm, root=0):
    """2A variant (BASELINE.json's "manual gather + broadcast"): rank-0 gather and mean as in
    ``sync_gradients_gather_scatter``, then ONE broadcast of the mean per parameter (RCCL runs
    it as a pipelined ring/tree over xGMI instead of world-1 point-to-point sends from rank 0)."""
    if not is_live(comm):
        return
    params = _params_with_grad(model)
    if comm.kind == "torch":
        for p in params:
            lst = comm.gather(p.grad, dst=root)
            if comm.rank == root:
                p.grad.copy_(torch.mean(torch.stack(lst), dim=0))
            comm.broadcast(p.grad, src=root)
        return
    from ..ops.common import native, stream_handle
    maxn = max(p.grad.numel() for p in params)
    staging = _staging(params[0].grad.device, comm.world, maxn) if comm.rank == root else None
    s = stream_handle()
    for p in params:
        g = p.grad
        n = g.numel()
        buf = staging[:comm.world * n].view(comm.world, n) if staging is not None else None
        comm.gather_into(g, buf, dst=root)
        if comm.rank == root:
            native().mean_ws(buf.data_ptr(), n, comm.world, g.data_ptr(), s)
        comm.broadcast(g, src=root)


_STAGING = {}


def _staging(device, world, maxn):
    key = (str(device), world)
    buf = _STAGING.get(key)
    if buf is None or buf.numel() < world * maxn:
        buf = torch.empty(world * maxn, dtype=torch.float32, device=device)
        _STAGING[key] = buf
    return buf


def sync_gradients_allreduce(model, comm):
    """2B: all_reduce(SUM) then divide by world size, one parameter at a time."""
    if not is_live(comm):
        return  # the mean over one replica is the gradient itself
    params = _params_with_grad(model)
    if comm.kind == "torch":
        for p in params:
            comm.all_reduce(p.grad, SUM)
            p.grad /= comm.world
        return
    from ..ops.common import native, stream_handle
    s = stream_handle()
    inv = 1.0 / comm.world
    for p in params:
        comm.all_reduce(p.grad, SUM)
        if comm.world > 1:
            native().scale(p.grad.data_ptr(), p.grad.numel(), inv, s)


STRATEGIES = {
    "gather_scatter": sync_gradients_gather_scatter,  # part 2A (reference: scatter)
    "gather_broadcast": sync_gradients_gather_broadcast,  # part 2A variant (gather + broadcast)
    "allreduce": sync_gradients_allreduce,            # part 2B
}
