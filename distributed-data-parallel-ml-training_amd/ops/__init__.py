"""Functional ops backed by the gfx950 HIP kernels in ``csrc/kernels``.

Each wrapper validates device / dtype / shape / contiguity on the host, then launches on the
current HIP stream (so the call can be captured into a hipGraph). There is no silent
fallback: on a GPU the native extension must be present (``ddp_amd._ext.load`` raises).
The CPU path of the framework uses plain ATen ops (it is the numerical oracle).
"""
from .common import native, ptr, stream_handle, grad_ready, register_grad_ready_hook, \
    clear_grad_ready_hooks  # noqa: F401
