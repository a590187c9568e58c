"""Seeding, device selection, JSON-lines metrics, checkpoints and a collective watchdog.

* seeding — reference: ``random.seed / torch.manual_seed / np.random.seed`` with seed 89395,
  called AFTER process-group init and BEFORE model construction so every rank builds identical
  initial weights (part1/main.py:14,115-117).
* checkpoints — the reference saves nothing; we save/load exactly the
  reference ``state_dict`` keys (``layers.N.weight`` ... ``fc1.bias``, fp32, no BN buffers),
  stripping/adding DDP's ``module.`` prefix, plus optional optimizer state.
* watchdog — the reference has no failure detection. A background thread
  checks that training makes progress and that RCCL reports no async error; on a hang or error
  it aborts the communicator and exits non-zero instead of blocking forever.
"""
import json
import os
import random
import sys
import threading
import time

import numpy as np
import torch


def seed_everything(seed):
    random.seed(seed)
    torch.manual_seed(seed)
    np.random.seed(seed)


def local_rank_of(rank=None):
    """GPU index for this process: LOCAL_RANK when a launcher (torchrun) set it, else the
    global rank — a reference-style launch (``main.py --num-nodes 8 --rank R`` once per GPU of
    one node, /root/reference/part3/main.py:29,36-40) has no LOCAL_RANK; ``pick_device`` then
    maps rank R to GPU ``R % device_count``."""
    if "LOCAL_RANK" in os.environ:
        return int(os.environ["LOCAL_RANK"])
    return int(rank) if rank is not None else 0


def pick_device(spec="auto", local_rank=None):
    if spec == "cpu":
        return torch.device("cpu")
    if spec in ("auto", "cuda") and torch.cuda.is_available():
        lr = local_rank if local_rank is not None else int(os.environ.get("LOCAL_RANK", "0"))
        n = torch.cuda.device_count()
        dev = torch.device("cuda", lr % max(n, 1))
        torch.cuda.set_device(dev)
        return dev
    if spec == "cuda":
        raise RuntimeError("--device cuda requested but no GPU is visible")
    return torch.device("cpu")


class MetricsSink:
    """Append-only JSON-lines metrics file (no-op when path is None)."""

    def __init__(self, path=None, rank=0):
        self.path, self.rank = path, rank

    def log(self, **kv):
        if not self.path:
            return
        kv.setdefault("ts", time.time())
        kv.setdefault("rank", self.rank)
        with open(self.path, "a") as f:
            f.write(json.dumps(kv) + "\n")


def _strip(sd):
    return {(k[len("module."):] if k.startswith("module.") else k): v for k, v in sd.items()}


def save_checkpoint(path, model, optimizer=None, extra=None):
    m = model.module if hasattr(model, "module") else model
    sd = {k: v.detach().float().cpu().contiguous() for k, v in m.state_dict().items()}
    obj = {"model": sd}
    if optimizer is not None:
        obj["optimizer"] = optimizer.state_dict()
    if extra:
        obj["extra"] = extra
    tmp = path + ".tmp"
    torch.save(obj, tmp)
    os.replace(tmp, path)


def load_checkpoint(path, model, optimizer=None, map_location="cpu"):
    obj = torch.load(path, map_location=map_location, weights_only=True)
    sd = obj["model"] if isinstance(obj, dict) and "model" in obj else obj
    m = model.module if hasattr(model, "module") else model
    with torch.no_grad():
        m.load_state_dict(_strip(sd))
    arena = getattr(next(m.parameters()), "_ddp_amd_arena", None)
    if arena is not None:
        arena.relink()
    if optimizer is not None and isinstance(obj, dict) and "optimizer" in obj:
        optimizer.load_state_dict(obj["optimizer"])
    return obj.get("extra") if isinstance(obj, dict) else None


def fault_point(rank, batch_idx):
    """Fault injection for the failure-detection tests:
    ``DDP_AMD_FAULT_INJECT=<rank>:<point>[:exit|hang]`` makes that rank die (``os._exit(17)``)
    or stop making progress (sleep forever) when it reaches that point: a batch index of the
    epoch, or a named point (``bench<k>``: bench.py start-up in fallback attempt k)."""
    spec = os.environ.get("DDP_AMD_FAULT_INJECT")
    if not spec:
        return
    parts = spec.split(":")
    if int(parts[0]) != int(rank) or parts[1] != str(batch_idx):
        return
    mode = parts[2] if len(parts) > 2 else "exit"
    print(f"[ddp_amd] fault injected on rank {rank} at batch {batch_idx}: {mode}",
          file=sys.stderr, flush=True)
    if mode == "hang":
        while True:
            time.sleep(3600)
    os._exit(17)


class Watchdog:
    """Abort the job when no progress is reported for ``timeout_s`` or RCCL reports an error."""

    def __init__(self, timeout_s=600.0, comm=None, poll_s=5.0, on_fail=None):
        self.timeout_s, self.comm, self.poll_s = timeout_s, comm, poll_s
        self.on_fail = on_fail
        self._last = time.monotonic()
        self._stop = threading.Event()
        self._thread = None
        self.failed = None

    def beat(self):
        self._last = time.monotonic()

    def _fail(self, why):
        self.failed = why
        print(f"[ddp_amd watchdog] {why}; aborting", file=sys.stderr, flush=True)
        if self.on_fail:
            self.on_fail(why)
            return
        try:
            if self.comm is not None and hasattr(self.comm, "abort"):
                self.comm.abort()
        finally:
            os._exit(3)

    def _run(self):
        while not self._stop.wait(self.poll_s):
            if self.comm is not None and hasattr(self.comm, "comm"):
                err = self.comm.comm.async_error()
                if err:
                    self._fail(f"RCCL async error {err}")
                    return
            if time.monotonic() - self._last > self.timeout_s:
                self._fail(f"no progress for {self.timeout_s:.0f}s (collective hang?)")
                return

    def start(self):
        self._thread = threading.Thread(target=self._run, daemon=True)
        self._thread.start()
        return self

    def stop(self):
        self._stop.set()
