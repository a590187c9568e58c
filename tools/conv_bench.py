#!/usr/bin/env python3
"""Per-layer implicit-GEMM conv timing on one MI355X (fwd / dgrad / wgrad, CUDA-event timed).

    python tools/conv_bench.py [--model vgg11|resnet50] [--batch B] [--reps R] [--json out.json]

Shapes are the model's own conv layers; every op is launched exactly as the training step does
(same tile selection, split-K and finish kernels). Prints us and achieved TFLOP/s per op.
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def vgg_layers(B):
    # (N, Cin_padded, H, W, K, R, stride, pad, Creal)
    cfg = [(3, 64, 32), (64, 128, 16), (128, 256, 8), (256, 256, 8), (256, 512, 4),
           (512, 512, 4), (512, 512, 2), (512, 512, 2)]
    out = []
    for cin, k, h in cfg:
        out.append((B, 8 if cin == 3 else cin, h, h, k, 3, 1, 1, cin))
    return out


def resnet_layers(B):
    out = [(B, 8, 224, 224, 64, 7, 2, 3, 3)]
    spatial = {64: 56, 128: 28, 256: 14, 512: 7}
    inp = 64
    for width, blocks, stride in [(64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)]:
        h_out = spatial[width]
        h_in = h_out * stride
        out.append((B, inp, h_in, h_in, width, 1, 1, 0, inp))
        out.append((B, width, h_in, h_in, width, 3, stride, 1, width))
        out.append((B, width, h_out, h_out, width * 4, 1, 1, 0, width))
        if stride != 1 or inp != width * 4:
            out.append((B, inp, h_in, h_in, width * 4, 1, stride, 0, inp))
        inp = width * 4
        if blocks > 1:  # a representative non-first block
            out.append((B, inp, h_out, h_out, width, 1, 1, 0, inp))
            if stride != 1:  # its 3x3 runs at stride 1 (the first block's is strided)
                out.append((B, width, h_out, h_out, width, 3, 1, 1, width))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="vgg11")
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    import torch
    import ddp_amd  # noqa: F401
    from ddp_amd.ops.layers import ConvBNActSpec, conv_forward, conv_backward
    dev = torch.device("cuda", 0)
    B = args.batch or (256 if args.model == "vgg11" else 64)
    layers = vgg_layers(B) if args.model == "vgg11" else resnet_layers(B)
    rows = []
    for (N, C, H, W, K, R, stride, pad, Cr) in layers:
        conv = torch.nn.Conv2d(Cr, K, R, stride, pad, bias=False).to(dev)
        conv.weight.data = conv.weight.data.contiguous(memory_format=torch.channels_last)
        spec = ConvBNActSpec(conv, None, cin_pad=C if C != Cr else None)
        spec.maybe_pack()
        P = (H + 2 * pad - R) // stride + 1
        x = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
        dz = torch.randn(N, P, P, K, device=dev).to(torch.bfloat16)
        dw = torch.zeros_like(conv.weight)
        stats = torch.zeros(16 * 2 * K, device=dev)
        flops = 2.0 * N * P * P * K * R * R * Cr
        ops = {"fwd": lambda: conv_forward(spec, x, None, stats),
               "wgrad": lambda: conv_backward(spec, x, dz, dw, False)}
        if C == Cr:
            ops["wgrad+dgrad"] = lambda: conv_backward(spec, x, dz, dw, True)
        res = {"shape": f"N{N} {Cr}->{K} {H}x{W} k{R} s{stride}"}
        for name, fn in ops.items():
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1000.0 / args.reps
            mult = 2 if name == "wgrad+dgrad" else 1
            res[name] = (round(us, 1), round(mult * flops / us / 1e6, 1))
        rows.append(res)
        print(res, flush=True)
    tot = {k: sum(r[k][0] for r in rows if k in r) for k in ("fwd", "wgrad", "wgrad+dgrad")}
    print("totals us:", {k: round(v, 1) for k, v in tot.items()})
    if args.json:
        with open(args.json, "w") as f:
            json.dump({"rows": rows, "totals_us": tot}, f, indent=1)


if __name__ == "__main__":
    main()
