#!/usr/bin/env python3
"""Per-step loss of the ResNet-50 training step, eager vs hipGraph replay (same process, same
weights, lr 0 so the weights never change): a captured step that reads memory it has not
written in the same replay shows up as replays whose loss differs from the eager steps.

    python tools/probes/resnet_graph_probe.py [--batch 256] [--steps 6] [--lr 0]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--lr", type=float, default=0.0)
    ap.add_argument("--model", default="resnet50")
    a = ap.parse_args()
    import torch
    import ddp_amd
    from ddp_amd.models import build
    from ddp_amd.engine import CrossEntropyLoss
    from ddp_amd.engine.step import TrainStep
    from ddp_amd.optim import FusedSGD
    from ddp_amd.data import SyntheticImageNet, SyntheticCIFAR10, DeviceLoader
    dev = torch.device("cuda", 0)
    torch.manual_seed(ddp_amd.SEED)
    resnet = a.model.startswith("resnet")
    ds = SyntheticImageNet(True, n=4 * a.batch) if resnet else SyntheticCIFAR10(True, n=4 * a.batch)
    loader = DeviceLoader(ds, a.batch, dev, 1, 0, train=True, cpad=8)
    model = build(a.model).to(dev)
    opt = FusedSGD(model.parameters(), lr=a.lr, momentum=0.9, weight_decay=1e-4)
    step = TrainStep(model, opt, CrossEntropyLoss(), loader, use_graph=True)
    eager = []
    for _ in range(a.steps):
        step.warmup(1)
        torch.cuda.synchronize()
        eager.append(step.pop_loss())
    print("eager ", " ".join(f"{v:.5f}" for v in eager), flush=True)
    step.capture()
    torch.cuda.synchronize()
    cap = step.pop_loss()  # the capture itself runs nothing
    graph = []
    arena = opt.arena

    def health(tag):
        bad = {k: int((~torch.isfinite(t)).sum()) for k, t in
               (("param", arena.data), ("grad", arena.grad), ("mom", opt.momentum_buffer))
               if t is not None}
        specs = [sp for sp in getattr(model, "fused_plan", lambda: [])() if hasattr(sp, "wc")]
        bad["wc"] = sum(int((~torch.isfinite(sp.wc.float())).sum()) for sp in specs)
        rs = [m for m in model.modules() if isinstance(m, torch.nn.BatchNorm2d)]
        bad["running"] = sum(int((~torch.isfinite(m.running_mean)).sum() +
                                 (~torch.isfinite(m.running_var)).sum()) for m in rs)
        print(f"  {tag}: non-finite {bad}", flush=True)
        if bad.get("param") and not getattr(health, "named", False):
            health.named = True
            names = [n for n, p in model.named_parameters() if not bool(torch.isfinite(p).all())]
            print(f"  non-finite parameters ({len(names)}): {names[:6]} ... {names[-6:]}", flush=True)

    for i in range(a.steps):
        step.step()
        torch.cuda.synchronize()
        graph.append(step.pop_loss())
        health(f"after graph step {i + 1} (loss {graph[-1]:.5f})")
    print("graph ", " ".join(f"{v:.5f}" for v in graph), f"(capture {cap:.5f})", flush=True)
    for _ in range(2):
        step.graph = None
        step.step()
        torch.cuda.synchronize()
        graph.append(step.pop_loss())
    print("eager after", " ".join(f"{v:.5f}" for v in graph[-2:]), flush=True)


if __name__ == "__main__":
    main()
