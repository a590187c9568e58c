#!/usr/bin/env python3
"""Config sweep of ResNet-50 b256's largest single GEMM dispatches (profiles/r5m_resnet50_b256.md):

* the stem weight gradient (7x7 / s2, 3 -> 64 channels, input padded to 8): one WGRAD GEMM
  M = 64, N = 7*7*8, K = 256*112*112 — split-K beyond the tuner's 64-way grid;
* the identity blocks' first 1x1 conv DGRAD in ACCUMULATE mode (dx = dgrad + first branch; the
  branch stored, or deferred as dy + ReLU bits), which the tuner timed only as a plain dgrad.

    python tools/probes/resnet_hot_probe.py [--reps 20]

Prints one line per (problem, tile, stages, splits), fastest first per problem, and the
cost-model / table choice. HIP events over back-to-back launches (each launch 100-500 us, so
the host launch floor does not matter here).
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
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    import torch
    import ddp_amd  # noqa: F401
    from ddp_amd.ops import common
    from ddp_amd.ops.common import native, ptr, workspace
    from ddp_amd.ops.layers import ConvBNActSpec
    n = native()
    dev = torch.device("cuda", 0)
    ws = workspace(dev)
    st = torch.cuda.current_stream().cuda_stream
    B = a.batch

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

    def sweep(label, fn, splits_list, tiles=range(8), modes_ok=lambda t: True):
        n.conv_force_tile(0, 0)
        auto = timeit(lambda: fn(0))
        res = []
        for t in tiles:
            if not modes_ok(t):
                continue
            tbm, tbn = (int(v) for v in TILES[t].split("x"))
            for nst in (2, 3, 4):
                if (tbm + tbn) * 64 * 2 * nst > 163840:
                    continue
                n.conv_force_tile(t + 1, nst)
                for s in splits_list:
                    try:
                        res.append((timeit(lambda: fn(s)), TILES[t], nst, s))
                    except RuntimeError as e:  # a config the launcher refuses
                        res.append((float("inf"), TILES[t], nst, f"{s} ({e})"))
        n.conv_force_tile(0, 0)
        res.sort(key=lambda r: r[0])
        print(f"\n## {label}: table / cost-model choice {auto:.1f} us\n", flush=True)
        print("| us | tile | stages | splits |\n|---|---|---|---|")
        for r in res[:12]:
            print(f"| {r[0]:.1f} | {r[1]} | {r[2]} | {r[3]} |", flush=True)

    # ---- stem WGRAD
    conv = torch.nn.Conv2d(3, 64, 7, 2, 3, bias=False).to(dev)
    conv.weight.data = conv.weight.data.contiguous(memory_format=torch.channels_last)
    spec = ConvBNActSpec(conv, None, cin_pad=8)
    spec.maybe_pack()
    x = torch.randn(B, 224, 224, 8, device=dev).to(torch.bfloat16)
    dz = torch.randn(B, 112, 112, 64, device=dev).to(torch.bfloat16)
    dw = torch.zeros_like(conv.weight)
    gw = spec.geom(B, 224, 224, common.weight_krsc(dw))
    # (split-K slabs: splits x 64 x 392 fp32 must fit the 32 Mi-element workspace)
    assert 1024 * 64 * 392 <= ws.numel()
    sweep(f"stem WGRAD b{B} (M 64, N 392, K {B * 112 * 112})",
          lambda s: n.conv_wgrad(gw, ptr(dz), ptr(x), ptr(dw), ptr(ws), ws.numel(), s, st),
          [64, 128, 256, 512, 1024], tiles=[1, 2, 3, 4], modes_ok=lambda t: t not in (5, 7))
    del x, dz, dw

    # ---- identity-block first 1x1 conv DGRAD, accumulate (stored and deferred first branch)
    for (Cin, K, H) in [(256, 64, 56), (512, 128, 28), (1024, 256, 14)]:
        conv = torch.nn.Conv2d(Cin, K, 1, 1, 0, bias=False).to(dev)
        conv.weight.data = conv.weight.data.contiguous(memory_format=torch.channels_last)
        spec = ConvBNActSpec(conv, None)
        spec.maybe_pack()
        g = spec.geom(B, H, H)
        dzk = torch.randn(B, H, H, K, device=dev).to(torch.bfloat16)
        dx = torch.randn(B, H, H, Cin, device=dev).to(torch.bfloat16)
        acc_dy = torch.randn_like(dx)
        mask = torch.randint(0, 256, (B, H, H, Cin // 8), dtype=torch.uint8, device=dev)
        ok = lambda t: t < 5  # noqa: E731  (DGRAD: the wide k-major tiles are refused)
        sweep(f"{Cin}->{K} {H}x{H} DGRAD plain",
              lambda s: n.conv_dgrad(g, ptr(dzk), ptr(spec.wc), ptr(dx), ptr(ws), ws.numel(), s, st),
              [1], modes_ok=ok)
        sweep(f"{Cin}->{K} {H}x{H} DGRAD accumulate (stored branch)",
              lambda s: n.conv_dgrad(g, ptr(dzk), ptr(spec.wc), ptr(dx), ptr(ws), ws.numel(), s, st,
                                     accumulate=1),
              [1], modes_ok=ok)
        sweep(f"{Cin}->{K} {H}x{H} DGRAD accumulate (deferred branch)",
              lambda s: n.conv_dgrad(g, ptr(dzk), ptr(spec.wc), ptr(dx), ptr(ws), ws.numel(), s, st,
                                     accumulate=1, acc_dy=ptr(acc_dy), acc_mask=ptr(mask)),
              [1], modes_ok=ok)
        del dzk, dx, acc_dy, mask


if __name__ == "__main__":
    main()
