#!/usr/bin/env python3
"""ResNet-50 b256 forward 1x1 convs that are write-bound in the step profile (the 64 -> 256
expansion over 56x56 writes 411 MB): time per (tile, stages) with and without the fused
BatchNorm statistics, and a plain write of the same bytes for the copy ceiling.

    python tools/probes/resnet_fwd_probe.py [--reps 20]

HIP events over back-to-back launches (each 50-200 us, far above the launch floor).
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)

TILES = ["128x128", "128x64", "64x128", "64x64", "256x64", "64x256", "256x128", "128x256"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--shapes", type=int, default=4, help="first N shapes only")
    a = ap.parse_args()
    import torch
    import ddp_amd  # noqa: F401
    from ddp_amd.ops.common import native, ptr, workspace
    from ddp_amd.ops.layers import ConvBNActSpec
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
        for _ in range(a.reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1000.0 / a.reps

    for (B, H, C, K, s) in [(256, 56, 64, 256, 1), (256, 56, 256, 64, 1), (256, 28, 128, 512, 1),
                            (256, 56, 64, 64, 1)][:a.shapes]:
        conv = torch.nn.Conv2d(C, K, 1, s, 0, bias=False).to(dev)
        spec = ConvBNActSpec(conv, None)
        spec.maybe_pack()
        x = torch.randn(B, H, H, C, device=dev).to(torch.bfloat16)
        P = H // s
        z = torch.empty(B, P, P, K, device=dev, dtype=torch.bfloat16)
        stats = torch.zeros(16 * 2 * K, device=dev)
        g = spec.geom(B, H, H)
        mb = (x.numel() + z.numel()) * 2 / 1e6
        copy_us = timeit(lambda: z.fill_(1.0))
        print(f"\n## 1x1 {C}->{K} {H}x{H} b{B}: reads {x.numel() * 2 / 1e6:.0f} MB, writes "
              f"{z.numel() * 2 / 1e6:.0f} MB; fill of the output alone {copy_us:.1f} us\n", flush=True)
        print("| tile | stages | stats us | no-stats us | GB/s (stats) |\n|---|---|---|---|---|")
        n.conv_force_tile(0, 0)
        auto_s = timeit(lambda: n.conv_fwd(g, ptr(x), ptr(spec.wc), 0, ptr(z), ptr(stats), ptr(ws),
                                           ws.numel(), 0, st))
        auto_n = timeit(lambda: n.conv_fwd(g, ptr(x), ptr(spec.wc), 0, ptr(z), 0, ptr(ws),
                                           ws.numel(), 0, st))
        print(f"| table | - | {auto_s:.1f} | {auto_n:.1f} | {mb / auto_s * 1e3:.0f} |", flush=True)
        for t in range(8):
            tbm, tbn = (int(v) for v in TILES[t].split("x"))
            for nst in (2, 3):
                if (tbm + tbn) * 64 * 2 * nst > 163840:
                    continue
                n.conv_force_tile(t + 1, nst)
                try:
                    ts = timeit(lambda: n.conv_fwd(g, ptr(x), ptr(spec.wc), 0, ptr(z), ptr(stats),
                                                   ptr(ws), ws.numel(), 0, st))
                    tn = timeit(lambda: n.conv_fwd(g, ptr(x), ptr(spec.wc), 0, ptr(z), 0, ptr(ws),
                                                   ws.numel(), 0, st))
                    print(f"| {TILES[t]} | {nst} | {ts:.1f} | {tn:.1f} | {mb / ts * 1e3:.0f} |", flush=True)
                except RuntimeError as e:
                    print(f"| {TILES[t]} | {nst} | refused ({e}) | | |")
        n.conv_force_tile(0, 0)
        del x, z


if __name__ == "__main__":
    main()
