#!/usr/bin/env python3
"""ResNet-50: does the fused bf16 GPU path follow the plain PyTorch (fp32, MIOpen) trajectory
over K SGD steps at the bench's hyper-parameters (lr 0.1, momentum 0.9, wd 1e-4)?

    python tools/resnet_traj_check.py [--batch 64] [--steps 20] [--lr 0.1]

Same initial weights, same batches (class-dependent Gaussian images, bf16-rounded). Prints
both loss sequences; a divergence of the fused path alone would point at a numerics bug, a
divergence of both at the configuration itself."""
import argparse
import copy
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F


def ref_forward(m, x):
    x = m.maxpool(m.relu(m.bn1(m.conv1(x))))
    for b in m.blocks():
        x = b(x)  # Bottleneck.forward: the ATen path
    return m.fc(torch.flatten(m.avgpool(x), 1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--res", type=int, default=224)
    args = ap.parse_args()
    import ddp_amd  # noqa: F401
    from ddp_amd.models.resnet import resnet50
    from ddp_amd.optim import FusedSGD
    from ddp_amd.engine import CrossEntropyLoss
    torch.manual_seed(0)
    base = resnet50()
    ref = copy.deepcopy(base).cuda()
    fus = copy.deepcopy(base).cuda()
    o_ref = torch.optim.SGD(ref.parameters(), lr=args.lr, momentum=0.9, weight_decay=1e-4)
    o_fus = FusedSGD(fus.parameters(), lr=args.lr, momentum=0.9, weight_decay=1e-4)
    crit = CrossEntropyLoss()
    g = torch.Generator(device="cuda").manual_seed(5)
    means = 0.25 * torch.randn(1000, 3, 1, 1, device="cuda", generator=g)
    lr_, lf_ = [], []
    for step in range(args.steps):
        y = torch.randint(0, 1000, (args.batch,), device="cuda", generator=g)
        x = torch.randn(args.batch, 3, args.res, args.res, device="cuda", generator=g) + means[y]
        x = x.to(torch.bfloat16).float()
        o_ref.zero_grad()
        lr = F.cross_entropy(ref_forward(ref, x), y)
        lr.backward()
        o_ref.step()
        o_fus.zero_grad()
        lf = crit(fus(x), y)
        lf.backward()
        o_fus.step()
        lr_.append(float(lr))
        lf_.append(float(lf))
        print(f"step {step:2d}  ref fp32 {lr_[-1]:8.4f}   fused bf16 {lf_[-1]:8.4f}", flush=True)
    pr = torch.cat([p.detach().reshape(-1) for p in ref.parameters()]).double()
    pf = torch.cat([p.detach().float().reshape(-1) for p in fus.parameters()]).double()
    print("param cosine", float(torch.dot(pr, pf) / (pr.norm() * pf.norm())))


if __name__ == "__main__":
    main()
