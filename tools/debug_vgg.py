"""Per-block numerics of the fused VGG path vs a bf16-emulating CPU oracle (debug tool)."""
import copy
import os
import sys

import torch
import torch.nn as nn
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))

from test_gpu_model import _Q, _QW  # noqa: E402


def rel(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-12))


def main():
    from ddp_amd.models import VGG11
    from ddp_amd.optim import FusedSGD
    from ddp_amd.ops.layers import conv_bn_act, linear_small, to_nhwc_input, cross_entropy
    torch.manual_seed(1)
    cpu = VGG11()
    gpu = copy.deepcopy(cpu).cuda()
    opt = FusedSGD(gpu.parameters(), lr=0.1)
    x = torch.randn(32, 3, 32, 32).to(torch.bfloat16).float()
    y = torch.randint(0, 10, (32,))

    # GPU, keeping block outputs
    def run_gpu():
        opt.zero_grad()
        hs = []
        h = to_nhwc_input(x.cuda(), 8)
        for spec in gpu.fused_plan():
            h = conv_bn_act(h, spec)
            h.retain_grad()
            hs.append(h)
        logits = linear_small(h.view(32, -1), gpu.fc1)
        loss = cross_entropy(logits, y.cuda())
        loss.backward()
        torch.cuda.synchronize()
        return loss, hs, opt.arena.grad.clone()

    l1, hs1, g1 = run_gpu()
    l2, hs2, g2 = run_gpu()
    print("determinism: loss diff", float(l1 - l2), "grad rel diff", rel(g2, g1))
    for i, (a, b) in enumerate(zip(hs1, hs2)):
        print(f"  block {i} dA rerun rel diff {rel(a.grad, b.grad):.2e}")

    # emulated CPU
    hs_e = []
    h = _Q.apply(x)
    mods = list(cpu.layers)
    i = 0
    while i < len(mods):
        conv, bn = mods[i], mods[i + 1]
        pool = i + 3 < len(mods) and isinstance(mods[i + 3], nn.MaxPool2d)
        z = _Q.apply(F.conv2d(h, _QW.apply(conv.weight), conv.bias, 1, 1))
        yy = F.relu(F.batch_norm(z, None, None, bn.weight, bn.bias, training=True, eps=bn.eps))
        if pool:
            yy = F.max_pool2d(yy, 2, 2)
        h = _Q.apply(yy)
        h.retain_grad()
        hs_e.append(h)
        i += 4 if pool else 3
    logits = cpu.fc1(h.view(32, -1))
    le = F.cross_entropy(logits, y)
    le.backward()
    print("loss gpu", float(l1), "emu", float(le))
    for i, (a, b) in enumerate(zip(hs1, hs_e)):
        fa = rel(a.detach().permute(0, 3, 1, 2).cpu(), b.detach())
        ba = rel(a.grad.permute(0, 3, 1, 2).cpu(), b.grad)
        print(f"  block {i}: fwd out rel {fa:.3e}   dA rel {ba:.3e}")


if __name__ == "__main__":
    main()
