#!/usr/bin/env python3
"""Measure every tile / split-K candidate of the implicit-GEMM conv for the training shapes and
write the winners to the launcher's tuning table (ops/conv_tuning.json).

    python tools/conv_tune.py [--out PATH] [--reps 30] [--quick]

Shapes: VGG-11 at per-GPU batch 256/128/64/32 (weak scaling and the reference's strong-scaling
split of 256 over 1/2/4/8 GPUs) and ResNet-50 at 64 and 256. For each GEMM problem (mode, M, N, K) every
tile (128x128, 128x64, 64x128, 64x64, and the big 256x64, 64x256, 256x128, 128x256) x LDS ring depth (2-4 stages) x split-K factor is launched exactly as the training step
launches it (same kernels, same finish passes), timed with HIP events, and the fastest is kept;
the cost-model choice is timed too and reported next to it. Like MIOpen's find-db, but for our
own kernels. Strided dgrad problems (several phase GEMMs) are tuned as a whole and the winner is
recorded for every phase.
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))

TILES = ["128x128", "128x64", "64x128", "64x64", "256x64", "64x256", "256x128", "128x256"]


def dgrad_phases(N, H, W, K, R, S, stride, pad):
    """(M, K) of each phase GEMM of a strided dgrad (mirrors ddp_conv_dgrad)."""
    if stride == 1:
        return [(N * H * W, R * S * K)]
    out = []
    for pa in range(stride):
        for pb in range(stride):
            r0, s0 = (pa + pad) % stride, (pb + pad) % stride
            Rt = (R - r0 + stride - 1) // stride if r0 < R else 0
            St = (S - s0 + stride - 1) // stride if s0 < S else 0
            Hp = (H - pa + stride - 1) // stride if pa < H else 0
            Wp = (W - pb + stride - 1) // stride if pb < W else 0
            if Rt * St == 0 or Hp * Wp == 0:
                continue
            out.append((N * Hp * Wp, Rt * St * K))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--quick", action="store_true", help="VGG-11 b256 only")
    ap.add_argument("--sets", default="all", choices=["all", "vgg", "resnet256"])
    ap.add_argument("--merge", default=None, help="existing table to extend (entries kept)")
    ap.add_argument("--modes", default="fwd,dgrad,wgrad",
                    help="GEMM kinds to tune (e.g. 'fwd': re-tune the forward entries only)")
    ap.add_argument("--pairs", action="store_true",
                    help="tune the backward pair launch (DGRAD+WGRAD split-K factors, or separate "
                         "launches) of the stride-1 layers instead (--pair-sets)")
    ap.add_argument("--pair-tiles", default="1,2,3,4,5",
                    type=lambda v: [int(t) for t in v.split(",")],
                    help="pair tiles to sweep (1 = 64x64, 2 = 128x128, 3 = 64x128, 4 = 128x64, "
                         "5 = 128x128 with 3 LDS stages)")
    ap.add_argument("--pair-sets", default="vgg11:32,64,128,256",
                    help="model:batches[;model:batches], e.g. 'resnet50:256'")
    args = ap.parse_args()
    if args.pairs:
        return tune_pairs(args)
    import torch
    import ddp_amd  # noqa: F401
    from ddp_amd.ops import common
    from ddp_amd.ops.common import native, ptr, workspace, TUNING_FILE
    from ddp_amd.ops.layers import ConvBNActSpec, bn_bwd_fuse_pays
    from conv_bench import vgg_layers, resnet_layers

    n = native()
    n.conv_tune_clear()  # time the cost-model choice without a previous table
    dev = torch.device("cuda", 0)
    ws = workspace(dev)
    st = torch.cuda.current_stream().cuda_stream
    ap_sets = {"quick": [("vgg11", 256)],
               "resnet256": [("resnet50", 256)],
               "vgg": [("vgg11", 256), ("vgg11", 128), ("vgg11", 64), ("vgg11", 32)],
               "all": [("vgg11", 256), ("vgg11", 128), ("vgg11", 64), ("vgg11", 32),
                       ("resnet50", 64), ("resnet50", 256)]}
    sets = ap_sets["quick" if args.quick else args.sets]
    entries, seen = [], set()
    saved_total = 0.0

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

    for model, B in sets:
        layers = vgg_layers(B) if model == "vgg11" else resnet_layers(B)
        prev_hw = None
        for (N, C, H, W, K, R, stride, pad, Cr) in layers:
            # VGG training dgrads carry the preceding block's fused BatchNorm-backward sums
            # (ops.layers BnBwdFuse): tune that variant. prev block's z is 2x larger if pooled.
            bn = None
            if (model == "vgg11" and prev_hw is not None and C == Cr
                    and bn_bwd_fuse_pays(H, W, prev_hw != H, N)):
                zh = prev_hw
                pz = torch.randn(N, zh, zh, C, device=dev).to(torch.bfloat16)
                pcoef = torch.rand(6 * C, device=dev)
                psums = torch.zeros(16 * 2 * C, device=dev)
                _keep = (pz, pcoef, psums)  # noqa: F841  (alive while timed)
                bn = (ptr(pz), ptr(pcoef), ptr(psums), int(zh != H), 1, zh, zh)
            prev_hw = H if model == "vgg11" else None
            conv = torch.nn.Conv2d(Cr, K, R, stride, pad, bias=False).to(dev)
            conv.weight.data = conv.weight.data.contiguous(memory_format=torch.channels_last)
            spec = ConvBNActSpec(conv, None, cin_pad=C if C != Cr else None)
            spec.maybe_pack()
            P = (H + 2 * pad - R) // stride + 1
            x = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
            z = torch.empty(N, P, P, K, device=dev, dtype=torch.bfloat16)
            dz = torch.randn(N, P, P, K, device=dev).to(torch.bfloat16)
            dx = torch.empty_like(x)
            dw = torch.zeros_like(conv.weight)
            stats = torch.zeros(16 * 2 * K, device=dev)
            g = spec.geom(N, H, W)
            gw = spec.geom(N, H, W, common.weight_krsc(dw))
            probs = []
            if C != 8:  # C = 8 input layers use the direct kernel forward (conv_smallk.hip)
                probs.append((0, [(N * P * P, K, R * R * C)],
                              lambda s: n.conv_fwd(g, ptr(x), ptr(spec.wc), 0, ptr(z), ptr(stats),
                                                   ptr(ws), ws.numel(), s, st)))
            if C == Cr:
                probs.append((1, [(m, C, k) for m, k in dgrad_phases(N, H, W, K, R, R, stride, pad)],
                              lambda s: n.conv_dgrad(g, ptr(dz), ptr(spec.wc), ptr(dx), ptr(ws),
                                                     ws.numel(), s, st, bn=bn)))
            probs.append((2, [(K, R * R * C, N * P * P)],
                          lambda s: n.conv_wgrad(gw, ptr(dz), ptr(x), ptr(dw), ptr(ws), ws.numel(),
                                                 s, st)))
            label = f"{model} N{N} {Cr}->{K} {H}x{W} k{R} s{stride}"
            for mode, gemms, fn in probs:
                key = (mode, tuple(gemms))
                if ["fwd", "dgrad", "wgrad"][mode] not in args.modes.split(","):
                    continue
                if key in seen:
                    continue
                seen.add(key)
                n.conv_force_tile(0, 0)
                auto_us = timeit(lambda: fn(0))
                best = (auto_us, None, None, None)
                M0, N0, K0 = gemms[0]
                ksteps = (K0 + 63) // 64
                for t in range(len(TILES)):
                    tbm, tbn = (int(v) for v in TILES[t].split("x"))
                    if mode == 1 and t >= 5:
                        # the 64x256 / 256x128 / 128x256 DGRAD configs return wrong dx (found by
                        # tests/test_gpu_kernels.py::test_conv_staged_epilogue with both epilogues)
                        # and were never selected; never let a sweep pick them
                        continue
                    for nst in (2, 3, 4):
                        if (tbm + tbn) * 64 * 2 * nst > 163840:
                            continue  # the ring would not fit the LDS (clamped by the launcher)
                        n.conv_force_tile(t + 1, nst)
                        for s in (1, 2, 3, 4, 6, 8, 12, 16, 24, 32, 48, 64):
                            if s > 1 and (ksteps // s < 2 or s * M0 * N0 > ws.numel()):
                                continue
                            us = timeit(lambda: fn(s))
                            if us < best[0] * 0.99:  # ties keep the simpler (earlier) config
                                best = (us, t, s, nst)
                n.conv_force_tile(0, 0)
                us, t, s, nst = best
                names = ["fwd", "dgrad", "wgrad"]
                if t is None:
                    print(f"{label:42s} {names[mode]:5s} auto {auto_us:7.1f} us (kept)", flush=True)
                    continue
                saved_total += auto_us - us
                print(f"{label:42s} {names[mode]:5s} auto {auto_us:7.1f} us -> {TILES[t]} "
                      f"split {s:2d} stages {nst} {us:7.1f} us", flush=True)
                for (M, Nn, Kk) in gemms:
                    entries.append({"mode": mode, "M": M, "N": Nn, "K": Kk, "tile": t,
                                    "splits": s, "stages": nst, "us": round(us, 2), "auto_us": round(auto_us, 2),
                                    "shape": label})
    table = {}
    if args.merge and os.path.exists(args.merge):
        with open(args.merge) as f:
            table = json.load(f)  # other sections (tap-reuse tables) are kept as they are
        old = table.get("entries", [])
        have = {(e["mode"], e["M"], e["N"], e["K"]) for e in entries}
        entries = [e for e in old if (e["mode"], e["M"], e["N"], e["K"]) not in have] + entries
    out = args.out or TUNING_FILE
    table.update({"device": torch.cuda.get_device_name(0), "reps": args.reps, "entries": entries})
    with open(out, "w") as f:
        json.dump(table, f, indent=1)
    print(f"wrote {len(entries)} entries to {out}; summed per-op saving {saved_total:.1f} us")


def tune_pairs(args):
    """Backward pair (ddp_conv_bwd_pair): for every stride-1 VGG-11 layer with a DGRAD, time the
    two separate launches, the policy's pair, and the forced pair over a grid of (DGRAD, WGRAD)
    split-K factors; record the winner as a mode-3 entry keyed by the DGRAD problem
    (tile = 1 pair with splits / stages = DGRAD / WGRAD splits, tile = 0 separate)."""
    import torch
    import ddp_amd  # noqa: F401
    from ddp_amd.ops import common
    from ddp_amd.ops.common import native, ptr, workspace, TUNING_FILE
    from ddp_amd.ops.layers import ConvBNActSpec, bn_bwd_fuse_pays
    from conv_bench import vgg_layers, resnet_layers

    n = native()
    dev = torch.device("cuda", 0)
    ws = workspace(dev)
    st = torch.cuda.current_stream().cuda_stream
    pair_mode = int(os.environ.get("DDP_AMD_BWD_PAIR", "3"))

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

    entries, saved, seen = [], 0.0, set()
    sets = []
    for item in args.pair_sets.split(";"):
        model, bs = item.split(":")
        sets += [(model, int(b)) for b in bs.split(",")]
    for model, B in sets:
        prev_hw = None
        layers = vgg_layers(B) if model == "vgg11" else resnet_layers(B)
        for (N, C, H, W, K, R, stride, pad, Cr) in layers:
            bn = None
            # (VGG: the preceding block's BN-backward sums ride in the dgrad epilogue; ResNet
            # keeps its separate reduce pass, ops/layers.py bn_bwd_fuse_pays)
            if (model == "vgg11" and prev_hw is not None and C == Cr
                    and bn_bwd_fuse_pays(H, W, prev_hw != H, N)):
                pz = torch.randn(N, prev_hw, prev_hw, C, device=dev).to(torch.bfloat16)
                pcoef = torch.rand(6 * C, device=dev)
                psums = torch.zeros(16 * 2 * C, device=dev)
                _keep = (pz, pcoef, psums)  # noqa: F841
                bn = (ptr(pz), ptr(pcoef), ptr(psums), int(prev_hw != H), 1, prev_hw, prev_hw)
            prev_hw = H
            if C != Cr or stride != 1 or (N, C, H, K, R) in seen:
                continue
            seen.add((N, C, H, K, R))
            conv = torch.nn.Conv2d(Cr, K, R, stride, pad, bias=False).to(dev)
            conv.weight.data = conv.weight.data.contiguous(memory_format=torch.channels_last)
            spec = ConvBNActSpec(conv, None)
            spec.maybe_pack()
            x = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
            dy = torch.randn(N, H, W, K, device=dev).to(torch.bfloat16)
            dx = torch.empty_like(x)
            dw = torch.zeros_like(conv.weight)
            gw = spec.geom(N, H, W, common.weight_krsc(dw))

            def call():
                n.conv_bwd_pair(gw, ptr(dy), ptr(spec.wc), ptr(dx), ptr(x), ptr(dw), ptr(ws),
                                ws.numel(), st, bn=bn)
            Md, Nd, Kd = N * H * W, C, R * R * K
            Mw, Nw, Kw = K, R * R * C, N * H * W
            n.conv_pair_force(0, 0, 0)
            n.conv_pair_mode(0, 0)
            sep = timeit(call)
            n.conv_pair_mode(pair_mode, 0)
            pol = timeit(call)
            best = (sep, 0, 1, 1)
            kd, kw = (Kd + 63) // 64, (Kw + 63) // 64
            # pair tiles (conv_igemm.hip kPairTiles): 1 = 64x64, 2 = 128x128, 3 = 64x128,
            # 4 = 128x64; a tile with fewer than ~64 work items before split-K is not tried
            tiles = [t for t, (bm, bn) in {1: (64, 64), 2: (128, 128), 3: (64, 128),
                                           4: (128, 64), 5: (128, 128)}.items()
                     if t in args.pair_tiles and
                     -(-Md // bm) * -(-Nd // bn) + -(-Mw // bm) * -(-Nw // bn) >= 64]
            for tile in tiles:
                for sd in (1, 2, 3, 4, 6, 8, 12, 16):
                    if sd > 1 and kd // sd < 2:
                        continue
                    for sw in (1, 2, 4, 6, 8, 12, 16, 24, 32, 48, 64, 96, 128):
                        if sw > 1 and kw // sw < 2:
                            continue
                        need = (sd * Md * Nd if sd > 1 else 0) + (sw * Mw * Nw if sw > 1 else 0) + 64
                        if need > ws.numel():
                            continue
                        n.conv_pair_force(sd, sw, tile)
                        us = timeit(call)
                        if us < best[0] * 0.99:
                            best = (us, tile, sd, sw)
            n.conv_pair_force(0, 0, 0)
            us, on, sd, sw = best
            ref = min(sep, pol)
            if pol <= us:  # the policy's own choice is (within noise) the best: no entry
                print(f"{model} N{N} {Cr}->{K} {H}x{W} k{R}: policy kept ({pol:.1f} us)", flush=True)
                continue
            saved += ref - us
            label = f"{model} N{N} {Cr}->{K} {H}x{W} k{R}"
            print(f"{label:32s} separate {sep:6.1f}  policy {pol:6.1f}  -> "
                  f"{f'pair tile {on}' if on else 'separate'} dg {sd:2d} wg {sw:3d} {us:6.1f} us",
                  flush=True)
            entries.append({"mode": 3, "M": Md, "N": Nd, "K": Kd, "tile": on, "splits": sd,
                            "stages": sw, "us": round(us, 2), "auto_us": round(pol, 2),
                            "shape": label + " bwd pair"})
    src = args.merge or TUNING_FILE
    table = {}
    if os.path.exists(src):
        with open(src) as f:
            table = json.load(f)  # other sections (tap-reuse tables) are kept as they are
    old = table.get("entries", [])
    have = {(e["mode"], e["M"], e["N"], e["K"]) for e in entries}
    entries = [e for e in old if (e["mode"], e["M"], e["N"], e["K"]) not in have] + entries
    out = args.out or TUNING_FILE
    table.update({"device": torch.cuda.get_device_name(0), "reps": args.reps, "entries": entries})
    with open(out, "w") as f:
        json.dump(table, f, indent=1)
    print(f"wrote {len(entries)} entries to {out}; pair saving vs policy {saved:.1f} us")


if __name__ == "__main__":
    main()
