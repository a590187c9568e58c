"""Flat parameter / gradient arenas.

All parameters of a model live in ONE contiguous fp32 buffer (``param.data`` becomes a view)
and all gradients in a second one (``param.grad`` is a view). This is what lets
* the optimizer update every tensor in a single kernel launch (optim/sgd.py),
* the DDP reducer all-reduce gradient buckets in place — a bucket is just a slice of the
  gradient arena in reverse parameter order, so there is no pack/unpack copy,
* rank-0 broadcast of the initial weights happen as one collective over the parameter arena.
Each tensor starts on a 64-element (256 B) boundary; padding elements stay zero forever.
"""
import torch

ALIGN = 64


class ParamArena:
    def __init__(self, params, device=None, align=ALIGN):
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
        self.data = torch.zeros(self.total, dtype=torch.float32, device=device)
        self.grad = torch.zeros(self.total, dtype=torch.float32, device=device)
        with torch.no_grad():
            for i, p in enumerate(plist):
                o, n = self.offsets[i], self.numels[i]
                self.data[o:o + n].copy_(p.detach().reshape(-1).float())
                p.data = self.data[o:o + n].view(p.shape)
                p.grad = self.grad[o:o + n].view(p.shape)
                p._ddp_amd_arena = self
                p._ddp_amd_index = i

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
                o, n = self.offsets[i], self.numels[i]
                if p.data.data_ptr() != self.data[o:o + n].data_ptr():
                    self.data[o:o + n].copy_(p.detach().reshape(-1))
                    p.data = self.data[o:o + n].view(p.shape)
                if p.grad is None or p.grad.data_ptr() != self.grad[o:o + n].data_ptr():
                    p.grad = self.grad[o:o + n].view(p.shape)


def arena_for(params, device=None):
    """Return the arena that already holds exactly these params, or build a new one."""
    plist = list(params)
    a = getattr(plist[0], "_ddp_amd_arena", None) if plist else None
    if a is not None and len(a.params) == len(plist) and all(x is y for x, y in zip(a.params, plist)):
        a.relink()
        return a
    return ParamArena(plist, device)
