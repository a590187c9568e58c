#!/usr/bin/env python3
"""Cost of the BatchNorm-statistics epilogue of the forward conv: time every ResNet-50 / VGG-11
forward conv with the stats reduction on (as trained) and off (stats=nullptr), same tile table.

    python tools/stat_probe.py [--model resnet50] [--batch 256]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default=None, help="substring of the shape label, e.g. '64-> 256'")
    ap.add_argument("--nostats", action="store_true", help="time only the stats-free launch")
    args = ap.parse_args()
    import torch
    import ddp_amd  # noqa: F401
    from ddp_amd.ops.common import native, ptr, workspace
    from ddp_amd.ops.layers import ConvBNActSpec
    from conv_bench import vgg_layers, resnet_layers
    n = native()
    dev = torch.device("cuda", 0)
    ws = workspace(dev)
    st = torch.cuda.current_stream().cuda_stream

    def timeit(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1000.0 / args.reps

    layers = vgg_layers(args.batch) if args.model == "vgg11" else resnet_layers(args.batch)
    seen, tot_on, tot_off = set(), 0.0, 0.0
    for (N, C, H, W, K, R, stride, pad, Cr) in layers:
        if C == 8 or (N, C, H, K, R, stride) in seen:
            continue
        seen.add((N, C, H, K, R, stride))
        label = f"N{N} {Cr:4d}->{K:4d} {H:3d}x{W:<3d} k{R} s{stride}"
        if args.only and args.only not in label:
            continue
        conv = torch.nn.Conv2d(Cr, K, R, stride, pad, bias=False).to(dev)
        conv.weight.data = conv.weight.data.contiguous(memory_format=torch.channels_last)
        spec = ConvBNActSpec(conv, None, cin_pad=C if C != Cr else None)
        spec.maybe_pack()
        P = (H + 2 * pad - R) // stride + 1
        x = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
        z = torch.empty(N, P, P, K, device=dev, dtype=torch.bfloat16)
        stats = torch.zeros(16 * 2 * K, device=dev)
        g = spec.geom(N, H, W)
        on = 0.0 if args.nostats else timeit(lambda: n.conv_fwd(g, ptr(x), ptr(spec.wc), 0, ptr(z), ptr(stats),
                                       ptr(ws), ws.numel(), 0, st))
        off = timeit(lambda: n.conv_fwd(g, ptr(x), ptr(spec.wc), 0, ptr(z), 0,
                                        ptr(ws), ws.numel(), 0, st))
        mb = (x.numel() + z.numel()) * 2 / 1e6
        gf = 2.0 * N * P * P * K * R * R * C / 1e9
        tot_on += on
        tot_off += off
        print(f"{label}  stats {on:7.1f} us  "
              f"none {off:7.1f} us  ({on - off:+6.1f})  {gf / max(on, off) * 1e3:6.0f} TF/s  "
              f"{mb / max(on, off):5.2f} TB/s", flush=True)
    print(f"total (unique shapes) stats {tot_on:.1f} us  none {tot_off:.1f} us")


if __name__ == "__main__":
    main()
