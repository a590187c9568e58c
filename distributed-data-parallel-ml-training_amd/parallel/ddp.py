"""Bucketed, backward-overlapped data parallelism (part 3).

Reference parity: ``torch.nn.parallel.DistributedDataParallel(model)`` with default settings
(part3/main.py:13,174):
* construction: verify parameter shapes across ranks, broadcast rank 0's parameters (and
  buffers) so every replica starts identical;
* every backward: gradients are averaged across ranks in buckets that are launched as soon as
  all their gradients exist, overlapping communication with the rest of the backward; the
  averaged gradients are in ``param.grad`` when ``loss.backward()`` returns.

MI355X design:
* gradients live in one flat fp32 arena (optim/arena.py); a bucket is a slice of it in reverse
  parameter order, so buckets are all-reduced in place with no pack/unpack copies;
* GPU: the native C++ ``Reducer`` (csrc/runtime/comm.cpp) over the host-only
  ``BucketScheduler`` (csrc/runtime/buckets.cpp; Python twin below) launches ncclAllReduce(avg)
  for each full bucket as soon as the fused backward kernels announce its last gradient
  (ops.common.grad_ready). EAGER backward passes issue it on a high-priority comm stream
  (event-gated), overlapped with the rest of the backward like torch DDP; a backward being
  CAPTURED into a hipGraph issues it inline on its own stream (a comm branch open across a
  captured backward runs 2.4x slower on ROCm 7, profiles/r1_comm_stream_study.md) — the captured
  multi-GPU step overlaps through engine/step.py SegmentedDDPStep instead;
* after iteration 0 the launch order is rebuilt from the observed gradient-ready order (torch
  DDP's bucket rebuild; buckets stay contiguous arena slices), broadcast from rank 0;
* CPU/Gloo: the same scheduler driven from post-accumulate-grad hooks with async all-reduce;
* bucket sizing for xGMI: 25 MiB + 1 MiB first by default (the reference's), or
  ``bucket_cap_mb="auto"``: from the all-reduce bus-bandwidth table (parallel/bucket_plan.py).
"""
import contextlib
import os

import torch
import torch.distributed as dist
import torch.nn as nn

from ..optim.arena import arena_for
from .comm import AVG, SUM, is_live


def plan_buckets(offsets, numels, elem_bytes, cap_bytes, cap_first_bytes):
    """Python twin of ddp_amd::plan_buckets (csrc/runtime/comm.cpp) — reverse parameter order."""
    out = []
    n = len(numels)
    end, start, nbytes = n, n, 0
    for p in range(n - 1, -1, -1):
        cap = cap_first_bytes if not out else cap_bytes
        pb = numels[p] * elem_bytes
        if start < end and nbytes + pb > cap:
            out.append((start, end, offsets[start], offsets[end - 1] + numels[end - 1] - offsets[start]))
            end, nbytes = start, 0
        start = p
        nbytes += pb
    if start < end:
        out.append((start, end, offsets[start], offsets[end - 1] + numels[end - 1] - offsets[start]))
    return out


class BucketScheduler:
    """Python twin of ddp_amd::BucketScheduler (csrc/runtime/buckets.h): per-bucket readiness
    counters and the launch order. ``mark(p)`` returns the buckets launchable now (in launch
    order: a bucket never overtakes an earlier one, so every rank issues collectives in the same
    order); ``finish()`` ends the backward pass, records the observed ready order and returns
    the remaining buckets; ``order_from_ready`` gives torch DDP's post-iteration-0 rebuild in
    this design's terms (bucket completion order; buckets stay contiguous arena slices)."""

    def __init__(self, buckets, n_params):
        self.buckets = [tuple(b) for b in buckets]
        self.bucket_of = [-1] * n_params
        for b, (s, e, _, _) in enumerate(self.buckets):
            if not 0 <= s < e <= n_params:
                raise RuntimeError(f"bucket {b} has a bad parameter range")
            for p in range(s, e):
                if self.bucket_of[p] != -1:
                    raise RuntimeError("parameter in two buckets")
                self.bucket_of[p] = b
        if any(b < 0 for b in self.bucket_of):
            raise RuntimeError("parameter in no bucket")
        self.order = list(range(len(self.buckets)))
        self._ready_order, self._launch_log = [], []
        self.prepare()

    def prepare(self):
        self.pending = [e - s for (s, e, _, _) in self.buckets]
        self.ready = [False] * len(self.buckets)
        self.seen = [False] * len(self.bucket_of)
        self.seq, self.log = [], []
        self.next_launch = 0
        self.marked = 0

    def _launchable(self):
        out = []
        while self.next_launch < len(self.order) and self.ready[self.order[self.next_launch]]:
            b = self.order[self.next_launch]
            self.next_launch += 1
            out.append(b)
            self.log.append((b, self.marked))
        return out

    def mark(self, p):
        if not 0 <= p < len(self.bucket_of):
            raise RuntimeError("bad param index")
        if self.seen[p]:
            raise RuntimeError("parameter marked ready twice in one backward")
        self.seen[p] = True
        self.seq.append(p)
        self.marked += 1
        b = self.bucket_of[p]
        self.pending[b] -= 1
        if self.pending[b] == 0:
            self.ready[b] = True
            return self._launchable()
        return []

    def finish(self):
        for b, r in enumerate(self.ready):
            if not r:
                raise RuntimeError(f"bucket {b} has parameters whose gradient was never produced "
                                   "(unused parameters are not supported)")
        rest = self._launchable()
        self._ready_order, self._launch_log = list(self.seq), list(self.log)
        self.prepare()
        return rest

    def launched(self):
        return self.next_launch

    def launch_order(self):
        return list(self.order)

    def set_launch_order(self, order):
        order = [int(b) for b in order]
        if sorted(order) != list(range(len(self.buckets))):
            raise RuntimeError("launch order is not a permutation of the buckets")
        if self.next_launch:
            raise RuntimeError("launch order changed during a backward")
        self.order = order

    def order_from_ready(self, seq):
        left = [e - s for (s, e, _, _) in self.buckets]
        done_at = [-1] * len(self.buckets)
        for i, p in enumerate(seq):
            b = self.bucket_of[p]
            left[b] -= 1
            if left[b] == 0:
                done_at[b] = i
        if any(d < 0 for d in done_at):
            raise RuntimeError("ready sequence does not complete every bucket")
        return sorted(range(len(self.buckets)), key=lambda b: done_at[b])

    def ready_order(self):
        return list(self._ready_order)

    def launch_log(self):
        return list(self._launch_log)


class _PyReducer:
    """Bucketed reducer for torch.distributed backends (Gloo on CPU): async all-reduce per bucket
    launched from post-accumulate-grad hooks (overlapped with the rest of the backward)."""

    def __init__(self, comm, arena, cap, cap_first, average, comm_dtype=torch.float32):
        self.comm, self.arena, self.average = comm, arena, average
        self.comm_dtype = comm_dtype
        self.sched = BucketScheduler(plan_buckets(arena.offsets, arena.numels, 4, cap, cap_first),
                                     len(arena.numels))
        self.buckets = self.sched.buckets
        self.works = []

    def prepare(self):
        self.sched.prepare()
        self.works = []

    def _launch(self, b):
        _, _, off, cnt = self.buckets[b]
        view = self.arena.grad[off:off + cnt]
        buf = view if self.comm_dtype == view.dtype else view.to(self.comm_dtype)
        self.works.append((view, buf, self.comm.all_reduce_async(buf)))

    def mark_ready(self, p):
        for b in self.sched.mark(p):
            self._launch(b)

    def finalize(self):
        for b in self.sched.finish():
            self._launch(b)
        for view, buf, w in self.works:
            w.wait()
            if buf is not view:
                view.copy_(buf)
            if self.average:
                view /= self.comm.world
        self.works = []

    # scheduler queries (same API as the native Reducer)
    def launched(self):
        return self.sched.launched()

    def launch_order(self):
        return self.sched.launch_order()

    def set_launch_order(self, order):
        self.sched.set_launch_order(order)

    def order_from_ready(self, seq):
        return self.sched.order_from_ready(seq)

    def ready_order(self):
        return self.sched.ready_order()

    def launch_log(self):
        return self.sched.launch_log()


class DistributedDataParallel(nn.Module):
    def __init__(self, module, comm, bucket_cap_mb=25.0, first_bucket_cap_mb=1.0,
                 broadcast_buffers=True, average=True, overlap=None, grad_comm_dtype="fp32",
                 captured=False, comm_table=None):
        super().__init__()
        self.module = module
        self.comm = comm
        self.broadcast_buffers = broadcast_buffers
        params = [p for p in module.parameters() if p.requires_grad]
        self.arena = arena_for(params)
        self.cuda = self.arena.data.is_cuda
        self._verify_param_shapes(params)
        self._sync_module_states()
        self.bucket_plan_reason = "explicit"
        if bucket_cap_mb == "auto" or first_bucket_cap_mb == "auto":
            # sized from the all-reduce bandwidth table for this world size (bucket_plan.py)
            from .bucket_plan import choose_bucket_caps
            wire = 2 if grad_comm_dtype == "bf16" else 4
            # ``captured``: the step will be captured into one hipGraph, whose bucket
            # collectives are issued inline (no overlap to buy): one bucket. ``comm_table``: a
            # table measured by the caller on this very communicator (bench.py start-up probe)
            # instead of comm_tuning.json
            cap_b, first_b, self.bucket_plan_reason = choose_bucket_caps(
                comm.world, self.arena.total * wire, overlap=not captured,
                dtype="bf16" if grad_comm_dtype == "bf16" else "fp32", table=comm_table)
            # the planner counts fp32 arena bytes
            cap, cap_first = cap_b * 4 // wire, first_b * 4 // wire
        else:
            cap = int(float(bucket_cap_mb) * (1 << 20))
            cap_first = int(float(first_bucket_cap_mb) * (1 << 20))
        self._index = {id(p): i for i, p in enumerate(self.arena.params)}
        self._in_backward = False
        self._sync_enabled = True
        # torch DDP rebuilds its buckets after iteration 0 from the observed gradient-ready
        # order (static_graph=False default). DDP_AMD_REBUILD_BUCKETS=0 keeps the plan order.
        self._iters = 0
        self._rebuilt = os.environ.get("DDP_AMD_REBUILD_BUCKETS", "1") == "0"
        self._flat_buffers = None
        self._stream = None
        if self.cuda:
            from ..ops.common import native, register_grad_ready_hook
            a = self.arena
            self.reducer = native().Reducer(comm.comm, a.grad.data_ptr(), list(a.offsets),
                                            list(a.numels), cap, cap_first, bool(average))
            self.buckets = [tuple(b) for b in self.reducer.buckets()]
            # Where the bucket collectives run (``overlap``; env DDP_AMD_COMM_OVERLAP=0/1 forces
            # it): None = auto — EAGER backward passes launch each full bucket on the comm stream
            # (event-gated), overlapped with the rest of the backward like the reference's DDP
            # (part3/main.py:174); a backward being CAPTURED into a hipGraph issues them inline
            # on its own stream instead: a captured comm branch that stays open across the
            # backward runs 2.4x slower on ROCm 7 (profiles/r1_comm_stream_study.md) — the
            # captured multi-GPU step overlaps through engine/step.py SegmentedDDPStep instead.
            if overlap is None and "DDP_AMD_COMM_OVERLAP" in os.environ:
                overlap = os.environ["DDP_AMD_COMM_OVERLAP"] == "1"
            self._overlap_mode = overlap  # None = auto
            if grad_comm_dtype not in ("fp32", "bf16"):
                raise ValueError("grad_comm_dtype must be 'fp32' or 'bf16'")
            self.reducer.set_overlap(True if overlap is None else bool(overlap))
            # world-1 stand-in collectives (one-GPU studies of the multi-GPU step):
            # DDP_AMD_EMULATE_COMM=N: N bucket-sized full-GPU passes per collective;
            # DDP_AMD_EMULATE_COMM_GBPS=G: a 32-CU kernel lasting bytes/G (RCCL-like footprint)
            emu = int(os.environ.get("DDP_AMD_EMULATE_COMM", "0"))
            gbps = float(os.environ.get("DDP_AMD_EMULATE_COMM_GBPS", "0"))
            self.reducer.set_emulate(emu > 0 or gbps > 0)
            self.reducer.set_emulate_passes(max(emu, 1))
            self.reducer.set_emulate_bw(gbps)
            # bf16 gradient communication (PyTorch's bf16_compress_hook): half the xGMI bytes;
            # the fp32 arena keeps the bf16-rounded average. Default fp32 = the reference.
            self.reducer.set_comm_dtype(1 if grad_comm_dtype == "bf16" else 0)
            # race-check mode (eager steps only — a host synchronise cannot be
            # captured): synchronise after every bucket collective, so a stream-ordering bug
            # shows up as a mismatch against the serial 2B path
            self.reducer.set_debug_sync(os.environ.get("DDP_AMD_DEBUG_SYNC", "0") == "1")
            self._hook = register_grad_ready_hook(self._on_grad_ready)
        else:
            self._overlap_mode = True  # async Gloo all-reduces launched from the hooks
            self.reducer = _PyReducer(comm, self.arena, cap, cap_first, average,
                                      torch.bfloat16 if grad_comm_dtype == "bf16" else torch.float32)
            self.buckets = self.reducer.buckets
            for p in self.arena.params:
                p.register_post_accumulate_grad_hook(self._on_accumulated)

    # ------------------------------------------------------------ construction-time sync
    def _verify_param_shapes(self, params):
        sig = torch.tensor([len(params)] + [s for p in params for s in p.shape] + [0] * 0,
                           dtype=torch.int64)
        if dist.is_initialized() and dist.get_world_size() > 1:
            n = torch.tensor([sig.numel()], dtype=torch.int64)
            sizes = [torch.zeros_like(n) for _ in range(dist.get_world_size())]
            dist.all_gather(sizes, n)
            if any(int(s) != int(n) for s in sizes):
                raise RuntimeError("DDP: parameter shapes differ across ranks")
            sigs = [torch.zeros_like(sig) for _ in range(dist.get_world_size())]
            dist.all_gather(sigs, sig)
            if any(not torch.equal(s, sig) for s in sigs):
                raise RuntimeError("DDP: parameter shapes differ across ranks")

    @torch.no_grad()
    def _sync_module_states(self):
        if not is_live(self.comm):
            return
        self.comm.broadcast(self.arena.data, 0)  # ONE coalesced broadcast of all parameters
        if self.broadcast_buffers:
            for b in self.module.buffers():
                self.comm.broadcast(b, 0)

    @torch.no_grad()
    def _flatten_buffers(self):
        """Re-point every module buffer (BatchNorm running statistics) at a view of one flat
        tensor per dtype, so the per-forward buffer broadcast is ONE collective per dtype instead
        of one per buffer (ResNet-50: 2 instead of 159)."""
        groups = {}
        for mod in self.module.modules():
            for name, b in mod._buffers.items():
                if b is not None:
                    groups.setdefault(b.dtype, []).append((mod, name, b))
        self._flat_buffers = []
        for dtype, items in groups.items():
            flat = torch.empty(sum(b.numel() for _, _, b in items), dtype=dtype,
                               device=items[0][2].device)
            off = 0
            for mod, name, b in items:
                view = flat[off:off + b.numel()].view_as(b)
                view.copy_(b)
                mod._buffers[name] = view
                off += b.numel()
            self._flat_buffers.append(flat)

    # ------------------------------------------------------------ per-step
    def _sync_buffers(self):
        if self.broadcast_buffers and is_live(self.comm) and torch.is_grad_enabled():
            if self._flat_buffers is None:
                self._flatten_buffers()
            with torch.no_grad():
                for flat in self._flat_buffers:
                    self.comm.broadcast(flat, 0)

    def _maybe_rebuild(self):
        """After the first synchronised backward: launch buckets in the order they completed
        (rank 0's observation, broadcast so every rank launches identically)."""
        if self._rebuilt or self._iters < 1 or not torch.is_grad_enabled():
            return
        if self.cuda and torch.cuda.is_current_stream_capturing():
            return
        self._rebuilt = True
        seq = list(self.reducer.ready_order())
        if not seq:
            return
        order = list(self.reducer.order_from_ready(seq))
        if self.comm.world > 1:
            # every rank must launch the buckets in the same order: take rank 0's observation
            # through the control plane. Without one that spans exactly this communicator's
            # ranks, locally observed orders could differ (hang / mixed-up buckets): keep the
            # plan order, which is identical everywhere by construction.
            if not (dist.is_available() and dist.is_initialized()
                    and dist.get_world_size() == self.comm.world):
                return
            box = [order]
            dist.broadcast_object_list(box, src=0)  # control plane (TCPStore / Gloo)
            order = box[0]
        self.reducer.set_launch_order(order)

    def forward(self, *args, **kwargs):
        self._maybe_rebuild()
        self._sync_buffers()
        return self.module(*args, **kwargs)

    def forward_loss(self, *args, **kwargs):
        """Fused forward + loss of the wrapped model (if it provides ``forward_loss``)."""
        self._maybe_rebuild()
        self._sync_buffers()
        return self.module.forward_loss(*args, **kwargs)

    @contextlib.contextmanager
    def no_sync(self):
        """Gradient accumulation without communication (torch DDP's ``no_sync``): backward
        passes inside the context accumulate into the gradient arena locally; the first backward
        after it all-reduces the accumulated gradients. (The reference has no accumulation —
        its report lists skipping synchronisations as future work.)"""
        prev, self._sync_enabled = self._sync_enabled, False
        try:
            yield
        finally:
            self._sync_enabled = prev

    def _queue_finalize(self):
        if not self._in_backward:
            self._in_backward = True
            torch.autograd.Variable._execution_engine.queue_callback(self._finalize)

    def _on_grad_ready(self, p, stream):
        i = self._index.get(id(p))
        if i is None or not self._sync_enabled:
            return
        if self._stream is None:
            # the backward's main stream (the first announcement comes from the classifier);
            # weight gradients may later be announced from the backward side stream — the
            # reducer then waits on both streams for the buckets they share
            self._stream = stream
            if self._overlap_mode is None:  # auto: comm stream when eager, inline when captured
                self.reducer.set_overlap(not torch.cuda.is_current_stream_capturing())
        self._queue_finalize()
        self.reducer.mark_ready(i, stream.cuda_stream)

    def _on_accumulated(self, p):
        i = self._index[id(p)]
        view = self.arena.shaped(self.arena.grad, i)
        if p.grad.data_ptr() != view.data_ptr():  # someone replaced .grad: fold it back
            view.copy_(p.grad)
            p.grad = view
        if not self._sync_enabled:
            return
        self._queue_finalize()
        self.reducer.mark_ready(i)

    def _finalize(self):
        self._in_backward = False
        self._iters += 1
        if self.cuda:
            stream, self._stream = self._stream, None
            self.reducer.finalize(stream.cuda_stream)
        else:
            self.reducer.finalize()

    def close(self):
        if self.cuda:
            from ..ops.common import clear_grad_ready_hooks
            clear_grad_ready_hooks(self._hook)

    # state_dict keys carry the reference's "module." prefix automatically (nn.Module nesting)


def replica_checksum(arena):
    """Exact integer checksum of the parameter arena (bit-level replica-consistency check)."""
    bits = arena.data.view(torch.int32).to(torch.int64)
    return int(bits.sum().item()), int((bits * torch.arange(bits.numel(), device=bits.device) % 1000003).sum().item())


def check_replicas(arena, world):
    """Return True iff every rank's parameters are bit-identical (control plane: Gloo)."""
    if world == 1 or not dist.is_initialized():
        return True
    c = torch.tensor(replica_checksum(arena), dtype=torch.int64)
    allc = [torch.zeros_like(c) for _ in range(world)]
    dist.all_gather(allc, c)
    return all(torch.equal(x, allc[0]) for x in allc)


__all__ = ["DistributedDataParallel", "BucketScheduler", "plan_buckets", "check_replicas", "replica_checksum", "SUM", "AVG"]
