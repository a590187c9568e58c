"""Shared helpers for the op wrappers: native handle, raw pointers, streams, grad-ready hooks."""
import torch

from .._ext import load as _load

_NATIVE = None


def native():
    global _NATIVE
    if _NATIVE is None:
        _NATIVE = _load()
    return _NATIVE


def ptr(t):
    """Raw device address of a tensor (0 for None)."""
    if t is None:
        return 0
    return t.data_ptr()


def stream_handle(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream


def check(t, dtype=None, shape=None, name="tensor"):
    if not t.is_cuda:
        raise ValueError(f"{name} must be a GPU tensor")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    if dtype is not None and t.dtype != dtype:
        raise ValueError(f"{name} must be {dtype}, got {t.dtype}")
    if shape is not None and tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name} shape {tuple(t.shape)} != expected {tuple(shape)}")
    return t


# ---------------------------------------------------------------- gradient-ready hooks
# Fused backward kernels write parameter gradients straight into the flat gradient arena
# (param.grad is a view into it) and return None to autograd. They announce completion here;
# the DDP reducer registers a hook to launch bucketed all-reduces as buckets fill up.
_HOOKS = []


def register_grad_ready_hook(fn):
    _HOOKS.append(fn)
    return fn


def clear_grad_ready_hooks(fn=None):
    if fn is None:
        _HOOKS.clear()
    elif fn in _HOOKS:
        _HOOKS.remove(fn)


def grad_ready(params):
    if not _HOOKS:
        return
    stream = torch.cuda.current_stream()
    for p in params:
        if p is None:
            continue
        for h in _HOOKS:
            h(p, stream)


def ensure_grad(p):
    """Gradient buffer for a parameter that fused kernels accumulate into."""
    if p.grad is None:
        p.grad = torch.zeros_like(p, memory_format=torch.contiguous_format)
    g = p.grad
    if not g.is_contiguous() or g.dtype != torch.float32:
        raise ValueError("fused kernels need contiguous fp32 .grad buffers")
    return g
