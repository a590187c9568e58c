"""roctx ranges around the phases of a training step.

The reference only times iterations with ``perf_counter_ns`` (part1/main.py:66,87). Here the
phases (data, forward, backward, sync, optimizer) can additionally be marked as roctx ranges so a
``rocprofv3 --marker-trace`` (or ``--kernel-trace --stats`` with markers) run attributes every
kernel to its phase. On a ROCm build of PyTorch ``torch.cuda.nvtx`` is backed by roctx.

Enabled with ``DDP_AMD_TRACE=1`` (or ``enable(True)``); disabled ranges cost one attribute test.
Ranges are host-side annotations: inside a captured hipGraph replay they are not re-emitted, so
trace eager steps (``--no-graph``) when attributing kernels to phases.
"""
import contextlib
import os

_ENABLED = os.environ.get("DDP_AMD_TRACE", "0") not in ("", "0")


def enable(on=True):
    global _ENABLED
    _ENABLED = bool(on)


def enabled():
    return _ENABLED


def _nvtx():
    try:
        import torch
        if torch.cuda.is_available():
            return torch.cuda.nvtx
    except Exception:
        pass
    return None


@contextlib.contextmanager
def trace_range(name):
    """``with trace_range("forward"): ...`` -> roctx push/pop when tracing is enabled."""
    nv = _nvtx() if _ENABLED else None
    if nv is None:
        yield
        return
    nv.range_push(name)
    try:
        yield
    finally:
        nv.range_pop()


def mark(name):
    """Instantaneous roctx marker."""
    nv = _nvtx() if _ENABLED else None
    if nv is not None:
        nv.mark(name)
