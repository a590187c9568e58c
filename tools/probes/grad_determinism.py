#!/usr/bin/env python3
"""Run the eager VGG-11 training step twice from one snapshot (parameters, momentum, data
cursor) and report, per parameter tensor, how much the two gradients differ: which layer's
backward is not run-to-run deterministic, and by how much.

    python tools/probes/grad_determinism.py [--batch 32] [--runs 3] [--hw 16,16,64]

``--hw`` sets ops.layers.BN_BWD_FUSE_MAX_HW per run (the threshold of the BatchNorm-backward
sums fused into the next dgrad's epilogue): a run with another threshold is then compared with
the run-to-run spread of the default ones.

SGD in the backward is switched off (the gradients stay in the arena)."""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
os.environ["DDP_AMD_SGD_IN_BWD"] = "0"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--hw", default="")
    a = ap.parse_args()
    import torch
    from ddp_amd.models import VGG11
    from ddp_amd.optim import FusedSGD
    from ddp_amd.data import SyntheticCIFAR10, DeviceLoader
    from ddp_amd.engine import TrainStep, CrossEntropyLoss
    from ddp_amd.ops import layers
    hws = [int(v) for v in a.hw.split(",")] if a.hw else [layers.BN_BWD_FUSE_MAX_HW] * a.runs
    a.runs = len(hws)
    torch.manual_seed(13)
    m = VGG11().cuda()
    opt = FusedSGD(m.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
    ld = DeviceLoader(SyntheticCIFAR10(True, n=max(256, a.batch)), a.batch, "cuda")
    st = TrainStep(m, opt, CrossEntropyLoss(), ld, sync=None)
    arena = opt.arena
    snap = (arena.data.clone(), opt.momentum_buffer.clone(), ld.cursor.clone())
    names = [n for n, _ in m.named_parameters()]
    params = [p for _, p in m.named_parameters()]
    grads = []
    for r in range(a.runs):
        layers.BN_BWD_FUSE_MAX_HW = hws[r]
        arena.data.copy_(snap[0])
        opt.momentum_buffer.copy_(snap[1])
        ld.cursor.copy_(snap[2])
        arena.grad.zero_()
        for sp in m.fused_plan():
            sp._packed_version = None
            sp.maybe_pack()
        torch.cuda.synchronize()
        # the step's fused SGD consumes and clears the gradient: capture it right after backward
        st.optimizer.step_orig = st.optimizer.step
        saved = {}

        def grab(*args, **kw):
            saved["g"] = [p.grad.detach().clone() if p.grad is not None else None for p in params]
            return st.optimizer.step_orig(*args, **kw)
        st.optimizer.step = grab
        st._body()
        torch.cuda.synchronize()
        st.optimizer.step = st.optimizer.step_orig
        grads.append(saved["g"])
    flat = [torch.cat([g.float().reshape(-1) for g in gr if g is not None]) for gr in grads]
    for r in range(a.runs):
        for q in range(r + 1, a.runs):
            d = float((flat[q] - flat[r]).norm() / flat[r].norm())
            print(f"runs {r} (hw {hws[r]}) vs {q} (hw {hws[q]}): whole-gradient relative difference {d:.3e}")
    print(f"batch {a.batch}: per-parameter max relative difference between runs (vs run 0)")
    for i, n in enumerate(names):
        g0 = grads[0][i]
        if g0 is None:
            continue
        rels = []
        for r in range(1, a.runs):
            d = (grads[r][i] - g0).float()
            rels.append(float(d.norm() / (g0.float().norm() + 1e-30)))
        print(f"  {n:40s} {tuple(g0.shape)!s:24s} |g| {float(g0.float().norm()):.3e}  "
              f"rel diff vs run 0 " + " ".join(f"{v:.3e}" for v in rels))


if __name__ == "__main__":
    main()
