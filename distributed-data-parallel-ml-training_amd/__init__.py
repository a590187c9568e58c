"""ddp_amd — an MI355X-native data-parallel training engine.

Capabilities mirror the CS744 reference (``ruc98/Distributed-Data-Parallel-ML-Training``):
VGG-family CNNs on CIFAR-10-shaped data trained with three gradient-synchronisation
strategies (rank-0 gather/mean/scatter, per-tensor all-reduce, bucketed overlapped DDP).

Layout:
    ops/       hand-written HIP/CDNA4 kernels wrapped as functional ops + autograd Functions
    models/    VGG-11/13/16/19 (reference-compatible state_dict keys) and ResNet-50
    parallel/  communicators (RCCL native, torch.distributed/gloo), sync strategies, DDP reducer
    data/      synthetic CIFAR-10 / ImageNet-shaped datasets, sharded sampler, fused augmentation
    engine/    train/eval loops, whole-step hipGraph capture
    utils/     CLI contract, seeding, timing/metrics, checkpoint, watchdog

Import as ``import ddp_amd`` (the top-level ``ddp_amd.py`` shim maps this directory).
"""
__version__ = "0.1.0"

SEED = 89395  # reference: part1/main.py:14


def native():
    """Return the compiled HIP/C++ extension module (raises if it is missing)."""
    from ._ext import load
    return load()
