"""Shared helpers for the op wrappers: native handle, raw pointers, streams, grad-ready hooks."""
import os

import torch

from .._ext import load as _load

_NATIVE = None
CONV_STAGES = 2  # LDS ring depth policy of untabulated conv GEMMs (2 = double buffering)
# backward-pair policy (conv_igemm.hip ddp_conv_pair_mode): 3 = pair when the measured pair
# table says so, or both problems pick the 64x64 tile, or the paired launch has <= 1024 items
BWD_PAIR_MODE, BWD_PAIR_ITEMS = 3, 1024


def native():
    global _NATIVE
    if _NATIVE is None:
        _NATIVE = _load()
        # (split-K always goes through fp32 slabs + a deterministic finish: the fp32-atomic
        # variants measured 6-60 % slower steps, profiles/r2_launch_reduction_ab.md, and were
        # removed in round 4)
        _NATIVE.conv_options(CONV_STAGES)
        _NATIVE.conv_pair_mode(BWD_PAIR_MODE, BWD_PAIR_ITEMS)
        load_conv_tuning(_NATIVE)
    return _NATIVE


TUNING_FILE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "conv_tuning.json")




def load_conv_tuning(n=None, path=None):
    """Load the measured conv tile / split-K table (tools/conv_tune.py) into the native launcher.
    DDP_AMD_CONV_TUNING=0 ignores it (cost-model choices only). Returns the number of entries."""
    import json
    n = n or native()
    n.conv_tune_clear()
    # (an empty DDP_AMD_CONV_TUNING_FILE means the shipped table, not "no table")
    path = path or os.environ.get("DDP_AMD_CONV_TUNING_FILE") or TUNING_FILE
    if os.environ.get("DDP_AMD_CONV_TUNING", "1") == "0" or not os.path.exists(path):
        return 0
    with open(path) as f:
        table = json.load(f)
    for e in table.get("entries", []):
        if int(e["mode"]) == 3 and "H" in e:  # backward pair of the layer with H x H outputs
            n.conv_pair_tune_set(int(e["M"]), int(e["N"]), int(e["K"]), int(e["H"]) ** 2,
                                 int(e["tile"]), int(e["splits"]), int(e.get("stages", 1)))
            continue
        n.conv_tune_set(int(e["mode"]), int(e["M"]), int(e["N"]), int(e["K"]), int(e["tile"]),
                        int(e["splits"]), int(e.get("stages", 0)))
    # tap-reuse 3x3 forward (conv_tr.hip, tools/conv_tune_tr.py): (M, K, C, H) -> (bm, bn,
    # splits); bm = 0 keeps the implicit-GEMM kernel for that layer
    n.conv_tr_set(-1, 0, 0, 0, 0, 0, 0, 0)
    for e in table.get("tr_entries", []):
        n.conv_tr_set(2, int(e["M"]), int(e["K"]), int(e["C"]), int(e["H"]), int(e["bm"]),
                      int(e["bn"]), int(e["splits"]), int(e.get("stages", 0)))
    return len(table.get("entries", [])) + len(table.get("tr_entries", []))


def weight_krsc(w):
    """1 if a 4-D fp32 weight (or weight gradient) is stored [K][R][S][C] (the GPU arena layout,
    optim/arena.py), 0 for the standard [K][C][R][S]. 1x1 kernels: both layouts coincide -> 0."""
    if w is None or w.dim() != 4 or w.shape[2] * w.shape[3] == 1 or w.shape[1] == 1:
        return 0
    return int(w.stride(1) == 1)


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


# ---------------------------------------------------------------- split-K slab workspace
# One persistent fp32 buffer per device, shared by every conv launch (they are stream-ordered).
# Allocated once, before any hipGraph capture, so captured graphs reference a static address.
WORKSPACE_ELEMS = 32 << 20  # 128 MiB of the 288 GB HBM
_WS = {}

def workspace(device):
    key = str(device)
    ws = _WS.get(key)
    if ws is None:
        ws = torch.empty(WORKSPACE_ELEMS, dtype=torch.float32, device=device)
        _WS[key] = ws
    return ws


# (Round 4 built and removed two more backward variants, both measured slower on every config:
# the apply-free BatchNorm backward whose dz the conv GEMMs computed while staging their A
# operand — VGG-11 b256 1.181 vs 0.852 ms, ResNet-50 35.89 vs 26.55 ms: the GEMMs staged z AND
# dy_bn and serialised their LDS ring on the rewrite — and the tap-reuse backward-data kernel,
# b256 0.898 vs 0.837 ms; profiles/r4d_ab.md, r4e_notes.md.)


# BatchNorm-backward sums of a Conv->BN->ReLU(->pool) block accumulated by the NEXT block's
# dgrad epilogue (BnBwdFuse, conv_igemm.hip): the block's backward skips its reduce pass.
# False: the separate reduce kernel (the tests' oracle).
BN_BWD_FUSE = True


# ---------------------------------------------------------------- per-step accumulator scratch
# Every fused layer owns fixed slices of one persistent fp32 buffer for the accumulators that
# must start at zero each step (BatchNorm statistics replicas, BN-backward sums). The model's
# forward zeroes the used prefix with ONE fill instead of one memset per layer and direction.
# Constraint: a forward must be followed by its backward before the next training forward.
_STAT_REPLICAS = None


def stat_replicas():
    """BatchNorm statistics replicas per accumulator (csrc/kernels/api.h kStatRep: 16, or one
    per block in the deterministic-statistics build)."""
    global _STAT_REPLICAS
    if _STAT_REPLICAS is None:
        _STAT_REPLICAS = int(native().stat_replicas())
    return _STAT_REPLICAS
SCRATCH_ELEMS = 8 << 20


class StepScratch:
    """Chunked: a process that builds many models (a test session) gets further chunks instead
    of running out; a single model lives in the first chunk, so its forward clears its
    accumulators with ONE fill (or none, when the loader's launch already did: claim_zero)."""

    def __init__(self, device):
        self.device = device
        self.chunks = [torch.zeros(SCRATCH_ELEMS, dtype=torch.float32, device=device)]
        self.used_in = [0]

    @property
    def buf(self):
        return self.chunks[0]

    @property
    def used(self):
        return self.used_in[0]

    def take(self, n):
        n = (n + 63) // 64 * 64
        off = self.used_in[-1]
        if off + n > self.chunks[-1].numel():
            self.chunks.append(torch.zeros(max(SCRATCH_ELEMS, n), dtype=torch.float32,
                                           device=self.device))
            self.used_in.append(0)
            off = 0
        self.used_in[-1] = off + n
        return self.chunks[-1][off:off + n]

    def take_transient(self, n):
        """A zeroed slice valid until the next zero(): consecutive calls within one forward get
        distinct slices (used for per-forward outputs such as the fused loss)."""
        if not hasattr(self, "_transient"):
            self._transient = self.take(256)
            self._tcur = 0
        if self._tcur + n > self._transient.numel():
            return torch.zeros(n, dtype=torch.float32, device=self.device)
        out = self._transient[self._tcur:self._tcur + n]
        self._tcur += n
        return out

    def claim_zero(self):
        """For a kernel that runs right before the next forward (the batch loader's augment
        launch): returns (pointer, count) of the region to clear and marks it cleared, so the
        forward's zero() skips its fill launch."""
        if len(self.chunks) != 1 or not self.used_in[0]:
            return 0, 0
        self._pre_zeroed = True
        return self.chunks[0].data_ptr(), self.used_in[0]

    def zero(self):
        if getattr(self, "_pre_zeroed", False):
            self._pre_zeroed = False  # cleared by the loader's launch for this forward
        else:
            for c, u in zip(self.chunks, self.used_in):
                if u:
                    c[:u].zero_()
        self._tcur = 0


_SCRATCH = {}


def step_scratch(device):
    key = str(device)
    s = _SCRATCH.get(key)
    if s is None:
        s = StepScratch(device)
        _SCRATCH[key] = s
    return s


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
    dense = g.is_contiguous() or (g.dim() == 4 and g.is_contiguous(memory_format=torch.channels_last))
    if not dense or g.dtype != torch.float32:
        raise ValueError("fused kernels need dense fp32 .grad buffers ([K][C][R][S] or [K][R][S][C])")
    return g
