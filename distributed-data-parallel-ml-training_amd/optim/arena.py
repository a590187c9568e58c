"""Flat parameter / gradient arenas.

All parameters of a model live in ONE contiguous fp32 buffer (``param.data`` becomes a view)
and all gradients in a second one (``param.grad`` is a view). This is what lets
* the optimizer update every tensor in a single kernel launch (optim/sgd.py),
* the DDP reducer all-reduce gradient buckets in place — a bucket is just a slice of the
  gradient arena in reverse parameter order, so there is no pack/unpack copy,
* rank-0 broadcast of the initial weights happen as one collective over the parameter arena.
Each tensor starts on a 64-element (256 B) boundary; padding elements stay zero forever.

Layout: on the GPU, 4-D conv weights are stored [K][R][S][C] ("KRSC", torch.channels_last for a
weight) — the layout the implicit-GEMM weight-gradient kernel produces natively, so its output
needs no transpose pass, and the bf16 forward operand is a plain conversion. ``param`` / ``grad``
keep their logical [K][C][R][S] shape (a permuted view), so state_dict keys, shapes and values are
exactly the reference's; only the strides differ.
"""
import torch

ALIGN = 64


class ParamArena:
    def __init__(self, params, device=None, align=ALIGN, krsc=None):
        seen, plist = set(), []
        for p in params:
            if id(p) not in seen:
                seen.add(id(p))
                plist.append(p)
        if not plist:
            raise ValueError("no parameters")
        device = device or plist[0].device
        self.params = plist
        self.offsets, self.numels = [], []
        off = 0
        for p in plist:
            self.offsets.append(off)
            self.numels.append(p.numel())
            off += (p.numel() + align - 1) // align * align
        self.total = off
        if krsc is None:
            krsc = torch.device(device).type == "cuda"
        self.krsc = [bool(krsc) and p.dim() == 4 for p in plist]
        self.data = torch.zeros(self.total, dtype=torch.float32, device=device)
        self.grad = torch.zeros(self.total, dtype=torch.float32, device=device)
        with torch.no_grad():
            for i, p in enumerate(plist):
                v = self.shaped(self.data, i)
                v.copy_(p.detach().float())
                p.data = v
                p.grad = self.shaped(self.grad, i)
                p._ddp_amd_arena = self
                p._ddp_amd_index = i

    def shaped(self, buf, i):
        """View of tensor i of a flat arena-shaped buffer (data, grad, momentum, ...) in the
        parameter's logical shape, honouring its storage layout."""
        o, n = self.offsets[i], self.numels[i]
        shape = self.params[i].shape
        flat = buf[o:o + n]
        if self.krsc[i]:
            K, C, R, S = shape
            return flat.view(K, R, S, C).permute(0, 3, 1, 2)
        return flat.view(shape)

    def index(self, p):
        return p._ddp_amd_index

    def param_view(self, i):
        return self.data[self.offsets[i]:self.offsets[i] + self.numels[i]]

    def grad_view(self, i):
        return self.grad[self.offsets[i]:self.offsets[i] + self.numels[i]]

    def zero_grad(self):
        self.grad.zero_()

    def relink(self):
        """Re-point .data/.grad at the arena (after e.g. load_state_dict replaced storages)."""
        with torch.no_grad():
            for i, p in enumerate(self.params):
                v = self.shaped(self.data, i)
                if p.data.data_ptr() != v.data_ptr() or p.data.stride() != v.stride():
                    v.copy_(p.detach())
                    p.data = v
                gv = self.shaped(self.grad, i)
                if p.grad is None or p.grad.data_ptr() != gv.data_ptr() or p.grad.stride() != gv.stride():
                    p.grad = gv


def arena_for(params, device=None):
    """Return the arena that already holds exactly these params, or build a new one."""
    plist = list(params)
    a = getattr(plist[0], "_ddp_amd_arena", None) if plist else None
    if a is not None and len(a.params) == len(plist) and all(x is y for x, y in zip(a.params, plist)):
        a.relink()
        return a
    return ParamArena(plist, device)
