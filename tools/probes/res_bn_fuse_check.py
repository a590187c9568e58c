#!/usr/bin/env python3
"""Numerics of the projection-shortcut BatchNorm fold (ops/layers.py RES_BN_FUSE, bn_act.hip
RBN) on ResNet-50, fold on vs off in one process:

1. one step's parameter gradients of each setting against plain PyTorch fp32 (same weights,
   same batch): relative error per parameter, worst 8 and the downsample parameters;
2. ``--repeats`` runs of the 10-step lr-0.01 trajectory of tests/test_gpu_resnet.py per
   setting: per-step relative loss differences against the fp32 run (run-to-run noise of the
   atomics-ordered bf16 path, to tell a numerics change from noise).

    python tools/probes/res_bn_fuse_check.py [--batch 32] [--repeats 3]
"""
import argparse
import copy
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))
import torch
import torch.nn.functional as F


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--repeats", type=int, default=3)
    a = ap.parse_args()
    import ddp_amd  # noqa: F401
    from ddp_amd.ops import layers
    from ddp_amd.models.resnet import resnet50
    from ddp_amd.optim import FusedSGD
    from ddp_amd.engine import CrossEntropyLoss
    from resnet_traj_check import ref_forward
    crit = CrossEntropyLoss()
    torch.manual_seed(0)
    base = resnet50()
    g = torch.Generator(device="cuda").manual_seed(5)
    means = 0.25 * torch.randn(1000, 3, 1, 1, device="cuda", generator=g)
    y = torch.randint(0, 1000, (a.batch,), device="cuda", generator=g)
    x = (torch.randn(a.batch, 3, 224, 224, device="cuda", generator=g) + means[y]).to(torch.bfloat16).float()
    ref = copy.deepcopy(base).cuda()
    F.cross_entropy(ref_forward(ref, x), y).backward()
    names = [n for n, _ in ref.named_parameters()]
    want = [p.grad.detach().float() for p in ref.parameters()]

    def grads(fuse):
        layers.RES_BN_FUSE = bool(fuse)
        m = copy.deepcopy(base).cuda()
        FusedSGD(m.parameters(), lr=0.0).zero_grad()
        crit(m(x), y).backward()
        torch.cuda.synchronize()
        return [p.grad.detach().float().clone() for p in m.parameters()]

    res = {}
    for fuse in (0, 1, 0, 1):
        gs = grads(fuse)
        errs = [float((gg - w).norm() / (w.norm() + 1e-30)) for gg, w in zip(gs, want)]
        res.setdefault(fuse, []).append(errs)
    print("## one-step gradient rel. error vs fp32 (two runs per setting)\n")
    print("| parameter | fold off | fold on |\n|---|---|---|")
    worst = sorted(range(len(names)), key=lambda i: -max(res[1][0][i], res[1][1][i]))[:8]
    ds = [i for i, n in enumerate(names) if "downsample" in n]
    for i in sorted(set(worst) | set(ds)):
        off = "/".join(f"{r[i]:.4f}" for r in res[0])
        on = "/".join(f"{r[i]:.4f}" for r in res[1])
        print(f"| {names[i]} | {off} | {on} |")
    for f in (0, 1):
        for r in res[f]:
            print(f"fold={f}: mean rel err {sum(r) / len(r):.5f}, max {max(r):.4f}")

    print("\n## 10-step trajectory (lr 0.01, batch %d): rel. loss diff vs fp32\n" % a.batch)
    for rep in range(a.repeats):
        for fuse in (0, 1):
            layers.RES_BN_FUSE = bool(fuse)
            torch.manual_seed(0)
            r = copy.deepcopy(base).cuda()
            f = copy.deepcopy(base).cuda()
            o_r = torch.optim.SGD(r.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
            o_f = FusedSGD(f.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
            g = torch.Generator(device="cuda").manual_seed(5)
            means = 0.25 * torch.randn(1000, 3, 1, 1, device="cuda", generator=g)
            rel = []
            for _ in range(10):
                yy = torch.randint(0, 1000, (a.batch,), device="cuda", generator=g)
                xx = (torch.randn(a.batch, 3, 224, 224, device="cuda", generator=g)
                      + means[yy]).to(torch.bfloat16).float()
                o_r.zero_grad()
                lr_ = F.cross_entropy(ref_forward(r, xx), yy)
                lr_.backward()
                o_r.step()
                o_f.zero_grad()
                lf = crit(f(xx), yy)
                lf.backward()
                o_f.step()
                rel.append(abs(float(lf) - float(lr_)) / float(lr_))
            print(f"rep {rep} fold={fuse}: max(first 6) {max(rel[:6]):.4f} mean {sum(rel) / 10:.4f} "
                  f"max {max(rel):.4f}  {[round(v, 4) for v in rel]}", flush=True)


if __name__ == "__main__":
    main()
