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

from ..utils.trace import trace_range


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
        import torch.distributed as dist
        mode = "global"
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            mode = "thread_local"
        with torch.cuda.graph(g, capture_error_mode=mode):
            self._body()
        self.graph = g

    def step(self):
        if self.graph is not None:
            self.graph.replay()
        else:
            self._body()

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
