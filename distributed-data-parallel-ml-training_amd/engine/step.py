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


class TrainStep:
    def __init__(self, model, optimizer, criterion, loader, sync=None, use_graph=True):
        self.model, self.optimizer, self.criterion, self.loader = model, optimizer, criterion, loader
        self.sync = sync
        self.use_graph = use_graph
        dev = loader.device
        self.loss_sum = torch.zeros((), dtype=torch.float32, device=dev)
        self._one = torch.ones((), dtype=torch.float32, device=dev)
        self.graph = None
        self.fused = self._fused_loss()
        self.fold_opt = bool(getattr(optimizer, "_fused", False)) and hasattr(loader, "cursor_advance")
        if self.fold_opt:
            optimizer.zero_grad()  # later steps get clean gradients from the previous step's launch

    def _fused_loss(self):
        """Use the model's fused classifier+loss when the criterion is the plain mean CE."""
        from .trainer import CrossEntropyLoss
        inner = getattr(self.model, "module", self.model)
        return (hasattr(self.model, "forward_loss") and hasattr(inner, "forward_loss")
                and type(self.criterion) is CrossEntropyLoss)

    def _body(self):
        if not self.fold_opt:
            self.optimizer.zero_grad()
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
                self.optimizer.step(zero_grad=True, counter=self.loader.cursor_advance())
            else:
                self.optimizer.step()
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
        if not self.use_graph:
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
        if self.fused:
            loss = self.model.forward_loss(x, y, acc=self.loss_sum)
        else:
            loss = self.criterion(self.model(x), y)
            self.loss_sum.add_(loss.detach())
        loss.backward(self._one)
        if self.sync is not None:
            self.sync(self.model)
        if self.fold_opt:
            self.optimizer.step(zero_grad=True)
        else:
            self.optimizer.step()

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
        self.graph = None  # divergent replicas under replay: run eagerly from now on
        return False

    def pop_loss(self):
        """Mean-free running loss sum since the last call (forces a device sync)."""
        v = float(self.loss_sum.item())
        self.loss_sum.zero_()
        return v


class SegmentedDDPStep(TrainStep):
    """DDP step whose late-layer gradient all-reduce overlaps the early layers' backward,
    without a comm branch inside a captured graph.

    Why: one captured graph whose comm-stream branch stays open across the backward runs 2.4-3x
    slower on ROCm 7 (profiles/r1_comm_stream_study.md: the graph executor spreads it over
    several hardware queues). Here the step is two single-stream graphs:

        g1 (main):  augment + forward + backward of the stages >= ``split`` -> flag_signal(S)
        eager:      comm stream: flag_wait(S) -> all-reduce bucket A (those stages' gradients,
                    VGG-11 split 4: 89% of the bytes; SECOND RCCL communicator) -> flag_signal(D)
        g2 (main):  backward of the stages < split -> all-reduce bucket B inline (DDP
                    communicator) -> flag_wait(D) -> fused SGD (+ grad clear, cursor advance)

    flag_signal / flag_wait (comm_util.hip) are an agent-scope release increment and a bounded
    one-wave spin (on timeout it records an error and returns) — cheaper than event edges
    between graph launches (~15 us idle per edge measured). Deadlock-free however HIP maps
    streams onto hardware queues: every wait's producer is enqueued before the wait in host
    order (the comm stream's wait follows g1's launch, g2's wait follows the all-reduce's
    launch), so a queue shared by producer and waiter holds the producer first. (A single-graph
    variant — comm work enqueued before the graph — measured faster but has the comm-side spin
    enqueued BEFORE its producer: on a shared hardware queue it deadlocks.)

    The DDP wrapper's own reducer is bypassed (``no_sync``); the arena is in parameter order, so
    bucket A is its tail. Models provide ``forward_loss_split`` / ``first_param_of_stage``
    (models/vgg.py). Measured with a 32-CU stand-in collective: profiles/r1_segmented_overlap.md.
    World size 1: the collectives are no-ops unless ``emulate`` > 0 (bucket-sized stand-in
    passes) or ``emulate_gbps`` > 0 (a 32-CU stand-in lasting bytes / emulate_gbps that then
    multiplies the bucket by ``emulate_scale``: an optimizer that did not wait would miss it).
    """

    WAIT_TIMEOUT_S = 100.0  # a device-side wait that exceeds this records an error and returns

    def __init__(self, ddp, optimizer, criterion, loader, split=4, emulate=0, emulate_gbps=0.0,
                 emulate_scale=1.0):
        super().__init__(ddp, optimizer, criterion, loader, sync=None, use_graph=True)
        inner = getattr(ddp, "module", None)
        if inner is None or not hasattr(inner, "forward_loss_split") or not self.fold_opt:
            raise ValueError("SegmentedDDPStep needs a DDP-wrapped model with forward_loss_split, "
                             "the fused optimizer and the device loader")
        self.ddp, self.split, self.emulate = ddp, int(split), int(emulate)
        self.emulate_gbps, self.emulate_scale = float(emulate_gbps), float(emulate_scale)
        arena = ddp.arena
        first = inner.first_param_of_stage(self.split)
        idx = next(i for i, p in enumerate(arena.params) if p is first)
        self.cut = arena.offsets[idx]
        self.total = arena.total
        self.comm_stream = torch.cuda.Stream()
        self.comm_a = None
        if is_live(ddp.comm):
            from ..parallel.comm import RcclCommunicator
            self.comm_a = RcclCommunicator(ddp.comm.rank, ddp.comm.world, ddp.comm.device,
                                           key="ddp_amd/rccl_uid_overlap", self_comm=True)
            # connect the communicator now: its first collective sets up the transports, which
            # must not count against the device-side wait timeout
            warm = torch.zeros(64, dtype=torch.float32, device=loader.device)
            self.comm_a.all_reduce(warm)
            torch.cuda.synchronize()
        # [0] = S (late backward done), [1] = D (bucket A reduced), [2], [3] = the waiters'
        # expected counts, [4] = error word
        self._flags = torch.zeros(8, dtype=torch.int32, device=loader.device)
        self.graphs = None
        self._h = self._h_leaf = None

    def _fp(self, i):
        return self._flags.data_ptr() + 4 * i

    def _allreduce(self, lo, hi, stream, comm):
        from ..ops.common import native
        from ..parallel.comm import AVG
        g = self.ddp.arena.grad
        n = hi - lo
        if comm is not None:
            comm.comm.all_reduce(g.data_ptr() + 4 * lo, n, 0, AVG, stream.cuda_stream)
        elif self.emulate_gbps > 0:  # timed 32-CU stand-in (comm_util.hip comm_standin)
            native().comm_standin(g.data_ptr() + 4 * lo, n, 32, 4.0 * n / (self.emulate_gbps * 1e3),
                                  self.emulate_scale, stream.cuda_stream)
        else:
            for _ in range(self.emulate):
                native().scale(g.data_ptr() + 4 * lo, n, 1.0, stream.cuda_stream)

    def _seg1(self):
        from ..ops.common import native
        self.ddp._sync_buffers()  # what DDP.forward would do (no-op without buffers / at world 1)
        with self.ddp.no_sync():
            with trace_range("data"):
                x, y = self.loader.fill(advance=False)
            with trace_range("forward"):
                loss, cuts = self.ddp.module.forward_loss_split(
                    x, y, self.split, acc=self.loss_sum, transient=True)
            with trace_range("backward_late"):
                loss.backward(self._one)
        self._h, self._h_leaf = cuts[0]
        native().flag_signal(self._fp(0), torch.cuda.current_stream().cuda_stream)

    def _comm_late(self):
        """Eager, between the graphs: wait S, bucket A on the comm stream, signal D."""
        from ..ops.common import native
        cs = self.comm_stream.cuda_stream
        native().flag_wait(self._fp(0), self._fp(2), self._fp(4), self.WAIT_TIMEOUT_S, cs)
        with trace_range("sync_late"):
            self._allreduce(self.cut, self.total, self.comm_stream, self.comm_a)
        native().flag_signal(self._fp(1), cs)

    def _seg2(self):
        from ..ops.common import native
        with self.ddp.no_sync():
            with trace_range("backward_early"):
                self._h.backward(self._h_leaf.grad)
        self._h = self._h_leaf = None
        main = torch.cuda.current_stream()
        with trace_range("sync_early"):  # bucket B, inline on the DDP communicator
            comm = self.ddp.comm if is_live(self.ddp.comm) else None
            self._allreduce(0, self.cut, main, comm)
        native().flag_wait(self._fp(1), self._fp(3), self._fp(4), self.WAIT_TIMEOUT_S,
                           main.cuda_stream)
        with trace_range("optimizer"):
            # a timed-out wait (error word set) skips the update: never apply gradients whose
            # bucket A was not averaged
            self.optimizer.step(zero_grad=True, counter=self.loader.cursor_advance(),
                                skip=self._fp(4))

    def _body(self):
        self._seg1()
        self._comm_late()
        self._seg2()

    def capture(self):
        torch.cuda.synchronize()
        self.check_error()
        mode = capture_mode()
        pool = torch.cuda.graph_pool_handle()  # activations of g1 are read by g2
        graphs = []
        for seg in (self._seg1, self._seg2):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=pool, capture_error_mode=mode):
                seg()
            graphs.append(g)
        self.graphs = graphs
        self.graph = graphs[0]  # "captured" marker for the shared helpers

    def step(self):
        if self.graph is None:  # never captured, or validate_distributed fell back to eager
            self._body()
            return
        self.graphs[0].replay()
        self._comm_late()
        self.graphs[1].replay()

    def check_error(self):
        """Raise if the device-side wait gave up (bucket A never completed within the timeout)."""
        if int(self._flags[4].item()) != 0:
            raise RuntimeError("SegmentedDDPStep: a device-side stream wait timed out "
                               f"(> {self.WAIT_TIMEOUT_S}s); the step's results are invalid")

    def validate_distributed(self, arena, world, timeout_s=120.0):
        ok = super().validate_distributed(arena, world, timeout_s)
        self.check_error()
        return ok

    def pop_loss(self):
        v = super().pop_loss()
        self.check_error()
        return v
