"""Whole-step hipGraph capture.

A training step on MI355X at the reference's global batch (256, or 32 per GPU at 8 GPUs) is
launch/latency bound: ~40 kernels forward+backward+optimizer at microsecond scale. Instead of a
tracing compiler we capture the ENTIRE step — on-device augmentation of the next batch, forward,
backward (whose fused kernels trigger the DDP bucket all-reduces on the comm stream through
events), the gradient sync of 2A/2B, and the fused SGD + weight re-pack — into one hipGraph and
replay it. Host cost per step becomes one graph launch.

Capture protocol: a few eager warm-up steps on a side stream (lazy allocations, autograd
structures), then ``torch.cuda.graph`` capture; replays are bit-identical to eager steps.
"""
import os

import torch

from ..parallel.comm import is_live
from ..utils.trace import trace_range


def capture_mode():
    """hipGraph capture mode: "thread_local" whenever RCCL communicators are live (several
    ranks, or a single-rank self communicator), else "global"."""
    import torch.distributed as dist
    from ..parallel import comm as _comm
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        return "thread_local"
    return "thread_local" if _comm.SELF_COMM_ACTIVE else "global"


def default_cuts(model_name, per_gpu_batch):
    """Backward cut points of the pipelined multi-GPU step (SegmentedDDPStep), from the one-GPU
    cut sweep with an 8-GPU-sized stand-in collective (profiles/r2_pipelined_ddp.md): VGG
    before stages 3 and 6 up to 128 images per GPU, 2 and 5 above; ResNet-50 before layer3 and
    layer4 (stages 8, 14)."""
    if model_name.startswith("resnet"):
        return "8,14"
    return "3,6" if per_gpu_batch <= 128 else "2,5"


def sgd_in_backward_ok(model):
    """May the optimizer step run inside the backward (TrainStep.opt_in_bwd)? Only when no
    gradient collective or stand-in reads the gradients: no live communicator, no emulated
    collective, and not switched off (DDP_AMD_SGD_IN_BWD=0)."""
    if os.environ.get("DDP_AMD_SGD_IN_BWD", "1") == "0":
        return False
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        return False  # gradients of a multi-rank job are reduced before any update
    if int(os.environ.get("DDP_AMD_EMULATE_COMM", "0")) > 0 or \
            float(os.environ.get("DDP_AMD_EMULATE_COMM_GBPS", "0")) > 0:
        return False
    comm = getattr(model, "comm", None)
    return comm is None or not is_live(comm)


class TrainStep:
    def __init__(self, model, optimizer, criterion, loader, sync=None, use_graph=True):
        self.model, self.optimizer, self.criterion, self.loader = model, optimizer, criterion, loader
        self.sync = sync
        self.use_graph = use_graph
        dev = loader.device
        self.loss_sum = torch.zeros((), dtype=torch.float32, device=dev)
        self._one = torch.ones((), dtype=torch.float32, device=dev)
        self.graph = None
        # set when a captured step was found to diverge across replicas (validate_distributed):
        # later capture() calls (a new epoch re-captures) keep running eager steps
        self.eager_only = False
        self.fused = self._fused_loss()
        self.fold_opt = bool(getattr(optimizer, "_fused", False)) and hasattr(loader, "cursor_advance")
        if self.fold_opt:
            optimizer.zero_grad()  # later steps get clean gradients from the previous step's launch
        # SGD in the backward: one GPU, no gradient collective (nothing reads a gradient between
        # its WGRAD finish and the update) -> each conv weight's update runs in the split-K
        # finish that completes its gradient; the step's SGD launch covers only the rest
        # (optim/sgd.py register_in_backward). DDP_AMD_SGD_IN_BWD=0 keeps the separate pass.
        self.opt_in_bwd = (self.fold_opt and sync is None and sgd_in_backward_ok(model)
                           and hasattr(optimizer, "register_in_backward"))

    def _fused_loss(self):
        """Use the model's fused classifier+loss when the criterion is the plain mean CE."""
        from .trainer import CrossEntropyLoss
        inner = getattr(self.model, "module", self.model)
        return (hasattr(self.model, "forward_loss") and hasattr(inner, "forward_loss")
                and type(self.criterion) is CrossEntropyLoss)

    def _body(self):
        if not self.fold_opt:
            self.optimizer.zero_grad()
        if self.opt_in_bwd:
            self.optimizer.register_in_backward()
        with trace_range("data"):
            x, y = self.loader.fill(advance=not self.fold_opt)
        with trace_range("forward"):
            if self.fused:
                # classifier + loss + loss meter in one kernel (no logits tensor, no extra adds)
                loss = self.model.forward_loss(x, y, acc=self.loss_sum, transient=True)
            else:
                loss = self.criterion(self.model(x), y)
        with trace_range("backward"):
            loss.backward(self._one)  # persistent ones: no fill kernel for the seed gradient
        if self.sync is not None:
            with trace_range("sync"):
                self.sync(self.model)
        with trace_range("optimizer"):
            if self.fold_opt:
                # the optimizer launch also clears the gradients for the next step and advances
                # the data cursor: no zero_grad fill, no counter kernel
                self.optimizer.step(zero_grad=True, counter=self.loader.cursor_advance(),
                                    fused_taken=self.opt_in_bwd)
            else:
                self.optimizer.step()
        if self.opt_in_bwd:
            self.optimizer.unregister_in_backward()
        if not self.fused:
            self.loss_sum.add_(loss.detach())

    def warmup(self, steps):
        """Eager steps on a side stream (also the fallback execution path)."""
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(steps):
                self._body()
        torch.cuda.current_stream().wait_stream(s)

    def capture(self):
        if not self.use_graph or self.eager_only:
            self.graph = None
            return
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        # Multi-GPU: RCCL keeps helper threads of its own; with the default "global" capture
        # mode any unsafe HIP call they make during the capture would invalidate it. Only the
        # capturing thread must stay capture-safe ("thread_local"); the replay is validated
        # against every replica afterwards (validate_distributed).
        mode = capture_mode()
        with torch.cuda.graph(g, capture_error_mode=mode):
            self._body()
        self.graph = g

    def step(self):
        if self.graph is not None:
            self.graph.replay()
        else:
            self._body()

    def tail_step(self, x, y):
        """One EAGER step on an explicit batch of any size (the epoch's partial last batch,
        engine/trainer.py train_model_graph): forward, backward, gradient sync (DDP buckets via
        the wrapper's reducer; 2A/2B via ``sync``) and the optimizer, on the same stream as the
        replays. Gradients are clear on entry when the optimizer launch clears them."""
        if not self.fold_opt:
            self.optimizer.zero_grad()
        if self.opt_in_bwd:
            self.optimizer.register_in_backward()
        if self.fused:
            loss = self.model.forward_loss(x, y, acc=self.loss_sum)
        else:
            loss = self.criterion(self.model(x), y)
            self.loss_sum.add_(loss.detach())
        loss.backward(self._one)
        if self.sync is not None:
            self.sync(self.model)
        if self.fold_opt:
            self.optimizer.step(zero_grad=True, fused_taken=self.opt_in_bwd)
        else:
            self.optimizer.step()
        if self.opt_in_bwd:
            self.optimizer.unregister_in_backward()

    def wait(self, timeout_s=None, poll_s=0.001):
        """Synchronise with the device, optionally bounded: returns False on timeout instead of
        blocking forever (a collective whose peer died would otherwise hang the process)."""
        if timeout_s is None:
            torch.cuda.synchronize()
            return True
        import time
        ev = torch.cuda.Event()
        ev.record()
        t0 = time.monotonic()
        while not ev.query():
            if time.monotonic() - t0 > timeout_s:
                return False
            time.sleep(poll_s)
        return True

    def validate_distributed(self, arena, world, timeout_s=120.0):
        """After capture on >1 ranks: replay once under a time limit and check that every
        replica is still bit-identical. Falls back to eager execution if the replicas diverged;
        raises if the replay did not finish (hung collective)."""
        from ..parallel.ddp import check_replicas
        if world <= 1:
            return True
        self.step()
        if not self.wait(timeout_s):
            raise RuntimeError(f"captured step did not finish within {timeout_s}s "
                               "(collective hang inside the hipGraph?)")
        if check_replicas(arena, world):
            return True
        self.graph = None  # divergent replicas under replay: run eagerly from now on ...
        self.eager_only = True  # ... including after a later capture() (next epoch)
        return False

    def pop_loss(self):
        """Mean-free running loss sum since the last call (forces a device sync)."""
        v = float(self.loss_sum.item())
        self.loss_sum.zero_()
        return v


class SegmentedDDPStep(TrainStep):
    """DDP step whose bucket all-reduces AND optimizer updates overlap the rest of the backward,
    without any comm branch inside a captured graph (VGG and ResNet; fp32 or bf16 gradients).

    Why: one captured graph whose comm-stream branch stays open across the backward runs 2.4-3x
    slower on ROCm 7 (profiles/r1_comm_stream_study.md: the graph executor spreads it over
    several hardware queues). The backward is therefore cut at the fused stages ``split``
    (models: ``forward_loss_split`` / ``first_param_of_stage``) into K+1 segments, each one
    single-stream graph on the main stream; bucket j is the arena slice of segment j's
    parameters (the arena is in parameter order, so bucket 0 = the LAST layers, whose gradients
    are ready first). Per step, host order:

        g[0] (main):  flag_wait(D) -> augment + forward + backward of segment 0 -> flag_signal(S)
        comm stream:  flag_wait(S) -> all-reduce bucket 0 -> fused SGD of bucket 0
        g[1] (main):  backward of segment 1 -> flag_signal(S)
        comm stream:  flag_wait(S) -> all-reduce bucket 1 -> fused SGD of bucket 1
        ...
        g[K] (main):  backward of segment K -> flag_signal(S)
        comm stream:  flag_wait(S) -> all-reduce bucket K -> fused SGD of bucket K (+ data
                      cursor advance) -> flag_signal(D)

    so each bucket's collective and its share of the optimizer run while the earlier layers are
    still back-propagating, and only the first layers' (small) bucket is exposed. The next
    step's forward waits for D (every parameter updated). flag_signal / flag_wait
    (comm_util.hip) are an agent-scope release increment and a bounded one-wave spin (on
    timeout it records an error word and returns; the optimizer launches skip the update when
    the word is set, so a timed-out step never applies unreduced gradients). Deadlock-free
    however HIP maps streams onto hardware queues: every wait's producer is enqueued before the
    wait in host order. The bucket collectives run eagerly on their OWN RCCL communicator
    (never mixed with graph-captured collectives of the DDP communicator, e.g. ResNet's
    BatchNorm-buffer broadcast inside g[0]); all of them sit on one stream, so they are
    serialised like the reference DDP's buckets (/root/reference/part3/main.py:174).

    The DDP wrapper's own reducer is bypassed (``no_sync``). World size 1 has no collective
    unless ``emulate`` > 0 (bucket-sized stand-in passes) or ``emulate_gbps`` > 0 (a 32-CU
    stand-in lasting bytes / emulate_gbps that then multiplies the bucket by ``emulate_scale``:
    an optimizer that did not wait would miss it). Measurements: profiles/r1_segmented_overlap.md
    (single cut, v4) and profiles/r2_pipelined_ddp.md.
    """

    WAIT_TIMEOUT_S = 100.0  # a device-side wait that exceeds this records an error and returns

    def __init__(self, ddp, optimizer, criterion, loader, split=4, emulate=0, emulate_gbps=0.0,
                 emulate_scale=1.0, grad_comm="fp32", zero=False, collectives=True,
                 update="allreduce", emulate_world=8, emulate_passes=1):
        super().__init__(ddp, optimizer, criterion, loader, sync=None, use_graph=True)
        # every bucket's update runs on the comm stream after its collective: never in the
        # backward (an emulated or single-rank collective still has to see the gradients)
        self.opt_in_bwd = False
        inner = getattr(ddp, "module", None)
        if inner is None or not hasattr(inner, "forward_loss_split") or not self.fold_opt:
            raise ValueError("SegmentedDDPStep needs a DDP-wrapped model with forward_loss_split, "
                             "the fused optimizer and the device loader")
        splits = [int(split)] if isinstance(split, (int, str)) else sorted(int(v) for v in split)
        self.ddp, self.splits, self.emulate = ddp, splits, int(emulate)
        self.split = splits[0] if len(splits) == 1 else splits
        self.emulate_gbps, self.emulate_scale = float(emulate_gbps), float(emulate_scale)
        # emulate_passes > 1: the stand-in collectives stream their bucket that many times,
        # paced over the modelled time (a live collective's memory traffic beside the backward)
        self.emulate_passes = max(1, int(emulate_passes))
        if grad_comm not in ("fp32", "bf16"):
            raise ValueError("grad_comm must be 'fp32' or 'bf16'")
        self.grad_comm = grad_comm
        arena = ddp.arena
        pidx = {id(p): i for i, p in enumerate(arena.params)}
        first = [pidx[id(inner.first_param_of_stage(sp))] for sp in splits]
        # buckets (param index ranges, arena element ranges), segment order = backward order
        bounds = [len(arena.params)] + first[::-1] + [0]
        self.buckets = []
        for j in range(len(bounds) - 1):
            i1, i0 = bounds[j], bounds[j + 1]
            lo = arena.offsets[i0]
            hi = arena.offsets[i1] if i1 < len(arena.params) else arena.total
            self.buckets.append(((i0, i1), (lo, hi)))
        self.cut = self.buckets[0][1][0]  # start of the last layers' bucket (tests)
        self.total = arena.total
        # The comm stream comes from HIP's HIGH-priority hardware-queue pool: normal-priority
        # streams share GPU_MAX_HW_QUEUES (4) queues round-robin, and with live RCCL
        # communicators (which create streams of their own) the comm stream landed on the main
        # stream's queue — every bucket then ran strictly between the segment graphs, 0 us
        # hidden; high priority: 76 of 120 us hidden (tools/overlap_probe.py,
        # profiles/r2_pipelined_ddp.md).
        self.comm_stream = torch.cuda.Stream(priority=-1)
        self.comm_a = None
        # collectives=False: no collective at all — no bucket all-reduce, no BatchNorm-buffer
        # broadcast (profile_stage_times: per-segment compute times of a cut-everywhere step on
        # a multi-rank job, state rolled back after; a rank that fails there cannot leave its
        # peers blocked inside a captured collective)
        self.sync_buffers = bool(collectives)
        if collectives and is_live(ddp.comm):
            from ..parallel.comm import RcclCommunicator
            self.comm_a = RcclCommunicator(ddp.comm.rank, ddp.comm.world, ddp.comm.device,
                                           key="ddp_amd/rccl_uid_overlap", self_comm=True)
            # connect the communicator now: its first collective sets up the transports, which
            # must not count against the device-side wait timeout
            warm = torch.zeros(64, dtype=torch.float32, device=loader.device)
            self.comm_a.all_reduce(warm)
            torch.cuda.synchronize()
        # Per-bucket update plan (parallel/cut_plan.py prices both):
        #   "ar"  all-reduce(avg) of the bucket's fp32 gradients -> replicated fused SGD
        #   "s16" reduce-scatter fp32 -> SGD on this rank's shard -> ONE grouped all-gather of the
        #         bf16 operand image + the small fp32 tensors (parallel/zero.py ShardedBf16Update)
        # ``update``: "allreduce" (all "ar"), "shard16" (all "s16"), or one code per bucket.
        # ``zero=True``: the fp32-master ZeRO-1 update of every bucket (ShardedUpdate).
        if isinstance(update, str):
            if update not in ("allreduce", "shard16"):
                raise ValueError("update must be 'allreduce', 'shard16' or a per-bucket list")
            update = ["s16" if update == "shard16" else "ar"] * len(self.buckets)
        update = list(update)
        if len(update) != len(self.buckets) or any(u not in ("ar", "s16") for u in update):
            raise ValueError(f"per-bucket update plan {update} does not match "
                             f"{len(self.buckets)} buckets")
        self.update = update
        self.zero = None
        self.shard16 = None
        if zero:
            if grad_comm != "fp32":
                raise ValueError("the sharded (ZeRO-1) update communicates fp32 gradients")
            from ..parallel.zero import ShardedUpdate
            self.zero = ShardedUpdate(arena, optimizer, self.comm_a or ddp.comm,
                                      [((i0, i1), (lo, hi)) for (i0, i1), (lo, hi) in self.buckets])
        elif "s16" in update:
            if grad_comm != "fp32":
                raise ValueError("the sharded bf16-gather update reduces fp32 gradients")
            from ..parallel.zero import ShardedBf16Update
            comm = self.comm_a or ddp.comm
            if hasattr(inner, "fused_plan"):
                inner.fused_plan()  # the operand copies (bf16 Wc) must exist to be re-pointed
            emu = None
            if comm.world == 1 and not is_live(comm) and (self.emulate or self.emulate_gbps > 0):
                emu = int(emulate_world)  # stand-in: shard as rank 0 of an N-GPU job
            self.shard16 = ShardedBf16Update(
                arena, optimizer, comm,
                [((i0, i1), (lo, hi)) for (i0, i1), (lo, hi) in self.buckets],
                which=[j for j, u in enumerate(update) if u == "s16"], emulate_world=emu)
        self._stage = None
        if grad_comm == "bf16":
            self._stage = torch.empty(arena.total, dtype=torch.bfloat16, device=loader.device)
        # [0] = S (segment backward done, counts up), [1] = D (step's updates done), [2], [3] =
        # the waiters' expected counts, [4] = error word, [5] = last-block-done ticket of the
        # launch that signals D. D starts at 1: the first step's forward has nothing to wait for.
        self._flags = torch.zeros(8, dtype=torch.int32, device=loader.device)
        self._flags[1] = 1
        self.graphs = None
        self._cuts = None
        # timing probe (tools/overlap_probe.py): list receiving (bucket, start, end) timing
        # events recorded on the comm stream around each bucket's collective + update
        self.probe = None

    def tail_step(self, x, y):
        """The epoch's partial last batch as one eager step. With a sharded update the masters
        and momentum are authoritative only on their shard owners and the replicated update of
        TrainStep.tail_step would diverge the replicas: refused (train full batches only, or
        use the all-reduce plan)."""
        if self.shard16 is not None or self.zero is not None:
            raise RuntimeError("SegmentedDDPStep: a partial batch needs the all-reduce update "
                               "(the sharded update keeps masters / momentum on shard owners)")
        torch.cuda.current_stream().wait_stream(self.comm_stream)
        super().tail_step(x, y)

    def _probe_event(self, stream):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(stream)
        return ev

    def _fp(self, i):
        return self._flags.data_ptr() + 4 * i

    def _allreduce(self, lo, hi, stream, comm):
        from ..ops.common import native
        from ..parallel.comm import AVG
        g = self.ddp.arena.grad
        n = hi - lo
        cs = stream.cuda_stream
        if comm is not None:
            if self._stage is not None:  # bf16 wire format: half the xGMI bytes
                sb = self._stage.data_ptr() + 2 * lo
                native().pack_bf16(g.data_ptr() + 4 * lo, n, sb, cs)
                comm.comm.all_reduce(sb, n, 1, AVG, cs)
                native().unpack_bf16(sb, n, g.data_ptr() + 4 * lo, cs)
            else:
                comm.comm.all_reduce(g.data_ptr() + 4 * lo, n, 0, AVG, cs)
        elif self.emulate_gbps > 0:  # timed 32-CU stand-in (comm_util.hip comm_standin)
            native().comm_standin(g.data_ptr() + 4 * lo, n, 32, 4.0 * n / (self.emulate_gbps * 1e3),
                                  self.emulate_scale, cs, self.emulate_passes)
        else:
            for _ in range(self.emulate):
                native().scale(g.data_ptr() + 4 * lo, n, 1.0, cs)

    def _seg_first(self):
        from ..ops.common import native
        main = torch.cuda.current_stream()
        native().flag_wait(self._fp(1), self._fp(3), self._fp(4), self.WAIT_TIMEOUT_S,
                           main.cuda_stream)
        if self.sync_buffers:
            self.ddp._sync_buffers()  # what DDP.forward would do (no-op without buffers / world 1)
        with self.ddp.no_sync():
            with trace_range("data"):
                x, y = self.loader.fill(advance=False)
            with trace_range("forward"):
                loss, cuts = self.ddp.module.forward_loss_split(
                    x, y, self.split, acc=self.loss_sum, transient=True)
            with trace_range("backward_seg0"):
                loss.backward(self._one)
        self._cuts = cuts
        native().flag_signal(self._fp(0), main.cuda_stream)

    def _seg(self, j):
        """Backward of segment j >= 1 (the stages before cut K-j+1)."""
        from ..ops.common import native
        h, leaf = self._cuts[len(self._cuts) - j]
        with self.ddp.no_sync():
            with trace_range(f"backward_seg{j}"):
                h.backward(leaf.grad)
        if j == len(self.buckets) - 1:
            self._cuts = None
        native().flag_signal(self._fp(0), torch.cuda.current_stream().cuda_stream)

    def _comm(self, j):
        """Eager, after segment j's graph: wait S, all-reduce bucket j, update its parameters
        (and after the last bucket: advance the data cursor, signal D)."""
        from ..ops.common import native
        cs = self.comm_stream
        native().flag_wait(self._fp(0), self._fp(2), self._fp(4), self.WAIT_TIMEOUT_S,
                           cs.cuda_stream)
        (i0, i1), (lo, hi) = self.buckets[j]
        last = j == len(self.buckets) - 1
        t0 = self._probe_event(cs) if self.probe is not None else None
        self._comm_body(j, cs, i0, i1, lo, hi, last)
        if t0 is not None:
            self.probe.append((j, t0, self._probe_event(cs)))

    def _standin(self, cs):
        """Timed stand-in for one collective of the sharded update (one GPU): a 32-CU pass
        lasting its modelled time at the all-reduce algorithm bandwidth ``emulate_gbps``; a
        reduce-scatter or an all-gather moves half an all-reduce's bytes per input byte."""
        from ..ops.common import native

        def run(kind, nbytes, ptr, n):
            if self.emulate_gbps > 0:
                us = 0.5 * nbytes / (self.emulate_gbps * 1e3)
                passes = self.emulate_passes
                if n == 0 and passes > 1:
                    # busy all-gather: stream the bucket's (already cleared) gradient slice, as
                    # many bytes as the bf16 all-gather moves (never the operand image itself)
                    (_, (lo, hi)) = self.buckets[self._standin_bucket]
                    ptr, n = self.ddp.arena.grad.data_ptr() + 4 * lo, (hi - lo) // 2
                native().comm_standin(ptr, n, 32, us, self.emulate_scale if kind != "all_gather" else 1.0,
                                      cs.cuda_stream, max(1, passes // 2))
            else:
                for _ in range(self.emulate):
                    if n:
                        native().scale(ptr, n, 1.0, cs.cuda_stream)
        return run

    def _comm_body(self, j, cs, i0, i1, lo, hi, last):
        from ..ops.common import native
        if self.shard16 is not None:
            if self.update[j] == "s16":
                self._standin_bucket = j
                with trace_range(f"shard16_update_bucket{j}"):
                    self.shard16.step(j, stream=cs, skip=self._fp(4),
                                      counter=self.loader.cursor_advance() if last else None,
                                      standin=self._standin(cs) if self.comm_a is None else None)
            else:
                with trace_range(f"sync_bucket{j}"):
                    self._allreduce(lo, hi, cs, self.comm_a)
                with trace_range(f"optimizer_bucket{j}"):
                    self.optimizer.step(zero_grad=True, params=(i0, i1), stream=cs,
                                        skip=self._fp(4),
                                        counter=self.loader.cursor_advance() if last else None)
            if last:  # small-tensor unpack + operand re-pack + signal D, one launch
                with trace_range("shard16_tail"):
                    self.shard16.tail(stream=cs, done=self._fp(5), signal=self._fp(1),
                                      skip=self._fp(4))
            return
        if self.zero is not None:
            with trace_range(f"zero_update_bucket{j}"):
                self.zero.step(j, stream=cs, skip=self._fp(4),
                               counter=self.loader.cursor_advance() if last else None)
            if last:
                native().flag_signal(self._fp(1), cs.cuda_stream)
            return
        with trace_range(f"sync_bucket{j}"):
            self._allreduce(lo, hi, cs, self.comm_a)
        with trace_range(f"optimizer_bucket{j}"):
            # a timed-out wait (error word set) skips the update: never apply gradients whose
            # bucket was not averaged
            # the last bucket's update launch also signals D (last-block-done ticket in
            # flags[5]): no separate signal launch on the critical comm stream
            self.optimizer.step(zero_grad=True, params=(i0, i1), stream=cs, skip=self._fp(4),
                                counter=self.loader.cursor_advance() if last else None,
                                signal=(self._fp(5), self._fp(1)) if last else None)

    def _segments(self):
        return [self._seg_first] + [(lambda j=j: self._seg(j)) for j in range(1, len(self.buckets))]

    def _body(self):
        for j, seg in enumerate(self._segments()):
            seg()
            self._comm(j)

    def capture(self):
        if self.eager_only:
            self.graph = self.graphs = None
            return
        torch.cuda.synchronize()
        self.check_error()
        mode = capture_mode()
        pool = torch.cuda.graph_pool_handle()  # activations of g[0] are read by later graphs
        graphs = []
        # each segment is its own single-stream graph (capturing runs no kernel: the flag
        # counters need no host-side bookkeeping)
        for seg in self._segments():
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=pool, capture_error_mode=mode):
                seg()
            graphs.append(g)
        self.graphs = graphs
        self.graph = graphs[0]  # "captured" marker for the shared helpers

    def step(self, seg_events=None):
        """One replayed step. ``seg_events``: list receiving a timing event recorded on the main
        stream before the first and after every segment graph (profile_stage_times)."""
        if self.graph is None:  # never captured, or validate_distributed fell back to eager
            self._body()
            return
        if seg_events is not None:
            seg_events.append(self._probe_event(torch.cuda.current_stream()))
        for j, g in enumerate(self.graphs):
            g.replay()
            if seg_events is not None:
                seg_events.append(self._probe_event(torch.cuda.current_stream()))
            self._comm(j)

    def check_error(self):
        """Raise if a device-side wait gave up (a bucket never completed within the timeout)."""
        if int(self._flags[4].item()) != 0:
            raise RuntimeError("SegmentedDDPStep: a device-side stream wait timed out "
                               f"(> {self.WAIT_TIMEOUT_S}s); the step's results are invalid")

    def sync_masters(self):
        """Make every rank's fp32 master weights complete (the sharded update keeps each
        operand tensor's master only on its shard owner): before check_replicas / state_dict."""
        if self.shard16 is not None:
            torch.cuda.current_stream().wait_stream(self.comm_stream)
            self.shard16.gather_masters()
            torch.cuda.synchronize()

    def validate_distributed(self, arena, world, timeout_s=120.0):
        if world <= 1:
            return True
        self.step()
        if not self.wait(timeout_s):
            raise RuntimeError(f"captured step did not finish within {timeout_s}s "
                               "(collective hang inside the hipGraph?)")
        self.check_error()
        self.sync_masters()
        from ..parallel.ddp import check_replicas
        if check_replicas(arena, world):
            return True
        self.graph = self.graphs = None
        self.eager_only = True
        return False

    def pop_loss(self):
        v = super().pop_loss()
        self.check_error()
        return v


def profile_stage_times(ddp, optimizer, criterion, loader, n_stages, reps=4):
    """Backward time of every fused stage at this per-GPU batch, measured on the device: a
    pipelined step cut before EVERY stage and without collectives is captured and replayed
    ``reps`` times with timing events between its segment graphs (the comm stream still runs
    each bucket's SGD, as in the real step). Segment j of that step is stage n_stages-1-j;
    stage n_stages-1's time also holds the forward, the classifier head and the data step.
    Parameters, momentum and the data cursor are rolled back afterwards (without collectives
    the replicas' updates would differ), so training continues from the same state on every
    rank. Returns a list of n_stages floats (us, median over reps). Feeds
    parallel/cut_plan.plan_cuts."""
    arena = ddp.arena
    snap = (arena.data.clone(), optimizer.momentum_buffer.clone(), loader.cursor.clone())
    # module buffers too (ResNet's BatchNorm running statistics): the profiling batches must
    # not leave extra updates behind
    bufs = [b for b in ddp.module.buffers()]
    bsnap = [b.clone() for b in bufs]
    st = SegmentedDDPStep(ddp, optimizer, criterion, loader, split=list(range(1, n_stages)),
                          collectives=False)
    try:
        st.warmup(1)
        st.capture()
        runs = []
        for r in range(reps + 1):
            evs = []
            st.step(seg_events=evs)
            torch.cuda.synchronize()
            if r:  # the first replay warms the graphs up
                runs.append([evs[i].elapsed_time(evs[i + 1]) * 1000.0 for i in range(len(evs) - 1)])
        st.check_error()
    finally:
        torch.cuda.synchronize()
        st.graphs = st.graph = None
        arena.data.copy_(snap[0])
        optimizer.momentum_buffer.copy_(snap[1])
        loader.cursor.copy_(snap[2])
        for b, v in zip(bufs, bsnap):
            b.copy_(v)
        arena.grad.zero_()
        optimizer.repack()
        torch.cuda.synchronize()
    per_seg = [sorted(col)[len(col) // 2] for col in zip(*runs)]
    return per_seg[::-1]  # segment j = stage n_stages-1-j
