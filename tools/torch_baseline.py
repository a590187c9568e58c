#!/usr/bin/env python3
"""Same-box PyTorch-ROCm baseline: plain PyTorch (MIOpen convolutions, hipBLASLt GEMMs, ATen
BatchNorm/ReLU/pool, torch.optim.SGD) for one training step of the reference ``VGG11()``
(/root/reference/part1/model.py:30-50, SGD(0.1, 0.9, 1e-4) from part1/main.py:124-125) and of
ResNet-50, timed eager and under ``torch.cuda.graph`` capture. No torch.compile (Triton).

bf16 autocast, channels_last, static synthetic inputs of the benchmark's shapes (no
augmentation inside the timed step, which favours the baseline slightly), fp32 master weights.

    python tools/torch_baseline.py --model vgg11 --batch 256 --steps 50
    python tools/torch_baseline.py --model resnet50 --batch 256 --steps 10

Prints one JSON line per (model, batch, mode).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def build_model(name):
    import torch.nn as nn
    from ddp_amd.models.vgg import VGG11
    from ddp_amd.models.resnet import resnet50

    if name == "vgg11":
        m = VGG11()

        class Plain(nn.Module):  # the reference forward, forced onto ATen on any device
            def __init__(self, m):
                super().__init__()
                self.m = m

            def forward(self, x):
                y = self.m.layers(x)
                return self.m.fc1(y.view(y.size(0), -1))
        return Plain(m), (3, 32, 32), 10
    if name == "resnet50":
        m = resnet50()

        class Plain(nn.Module):  # torchvision's ResNet.forward on ATen
            def __init__(self, m):
                super().__init__()
                self.m = m

            def forward(self, x):
                import torch
                m = self.m
                x = m.maxpool(m.relu(m.bn1(m.conv1(x))))
                x = m.layer4(m.layer3(m.layer2(m.layer1(x))))
                return m.fc(torch.flatten(m.avgpool(x), 1))
        return Plain(m), (3, 224, 224), 1000
    raise SystemExit(f"unknown model {name}")


def run(name, batch, steps, warmup, mode, lr):
    import torch
    torch.manual_seed(89395)
    dev = torch.device("cuda", 0)
    model, shape, ncls = build_model(name)
    model = model.to(dev).to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(model.parameters(), lr=lr, momentum=0.9, weight_decay=1e-4,
                          foreach=True)
    crit = torch.nn.CrossEntropyLoss()
    x = torch.randn(batch, *shape, device=dev).to(memory_format=torch.channels_last)
    y = torch.randint(0, ncls, (batch,), device=dev)

    def step():
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
            loss = crit(model(x), y)
        loss.backward()
        opt.step()
        return loss

    if mode == "graph":
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(3):
                step()
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        opt.zero_grad(set_to_none=True)
        with torch.cuda.graph(g):
            with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
                static_loss = crit(model(x), y)
            static_loss.backward()
            opt.step()
        fn = g.replay
    else:
        fn = step
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    out = {"model": name, "batch": batch, "mode": mode, "ms_per_step": round(dt * 1e3, 4),
           "images_per_s": round(batch / dt, 1), "stack": "pytorch-rocm (MIOpen/hipBLASLt, "
           "bf16 autocast, channels_last, torch.optim.SGD foreach)",
           "torch": torch.__version__}
    print(json.dumps(out), flush=True)
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--model", default="vgg11")
    p.add_argument("--batch", type=int, nargs="+", default=[256])
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--modes", nargs="+", default=["eager", "graph"])
    p.add_argument("--lr", type=float, default=None)
    a = p.parse_args()
    lr = a.lr if a.lr is not None else (0.01 if a.model.startswith("resnet") else 0.1)
    for b in a.batch:
        for m in a.modes:
            try:
                run(a.model, b, a.steps, a.warmup, m, lr)
            except Exception as e:  # keep the other configurations measurable
                print(json.dumps({"model": a.model, "batch": b, "mode": m, "error": repr(e)}),
                      flush=True)


if __name__ == "__main__":
    main()
