#!/usr/bin/env python3
"""How far is each VGG-11 conv from what the platform libraries reach on the same shapes?

Per layer (forward only, bf16, back-to-back launches, CUDA-event timed):
  ours    conv_forward (implicit-GEMM MFMA kernel, BN statistics in the epilogue, as trained)
  miopen  torch conv2d, channels_last bf16 (MIOpen)
  gemm    torch.matmul of the im2col-equivalent GEMM [M, 9C] x [9C, K] (hipBLASLt), i.e. the
          same FLOPs with a materialised, perfectly streamed A operand (an upper bound on what
          a GEMM library does with these dimensions)

    python tools/probes/gemm_ceiling.py --batch 256 32
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))


def timeit(fn, reps=30):
    import torch
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, nargs="+", default=[256, 32])
    a = ap.parse_args()
    import torch
    import ddp_amd  # noqa: F401
    from ddp_amd.ops.layers import ConvBNActSpec, conv_forward
    from conv_bench import vgg_layers
    dev = torch.device("cuda", 0)
    for B in a.batch:
        tot = {"ours": 0.0, "miopen": 0.0, "gemm": 0.0}
        for (N, C, H, W, K, R, stride, pad, Cr) in vgg_layers(B):
            conv = torch.nn.Conv2d(Cr, K, R, stride, pad, bias=False).to(dev)
            conv.weight.data = conv.weight.data.contiguous(memory_format=torch.channels_last)
            spec = ConvBNActSpec(conv, None, cin_pad=C if C != Cr else None)
            spec.maybe_pack()
            x = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
            stats = torch.zeros(16 * 2 * K, device=dev)
            flops = 2.0 * N * H * W * K * 9 * Cr
            xt = torch.randn(N, Cr, H, W, device=dev, dtype=torch.bfloat16).contiguous(
                memory_format=torch.channels_last)
            cw = conv.weight.detach().to(torch.bfloat16)
            A = torch.randn(N * H * W, 9 * Cr, device=dev, dtype=torch.bfloat16)
            Bm = torch.randn(9 * Cr, K, device=dev, dtype=torch.bfloat16)
            r = {"batch": B, "shape": f"{Cr}->{K} {H}x{W}",
                 "ours": timeit(lambda: conv_forward(spec, x, None, stats)),
                 "miopen": timeit(lambda: torch.nn.functional.conv2d(xt, cw, None, 1, 1)),
                 "gemm": timeit(lambda: torch.matmul(A, Bm))}
            for k in tot:
                tot[k] += r[k]
                r[k + "_tflops"] = round(flops / r[k] / 1e6, 1)
                r[k] = round(r[k], 2)
            print(json.dumps(r), flush=True)
        print(json.dumps({"batch": B, "totals_us": {k: round(v, 1) for k, v in tot.items()}}),
              flush=True)


if __name__ == "__main__":
    main()
