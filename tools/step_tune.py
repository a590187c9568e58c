#!/usr/bin/env python3
"""Backward-pair table tuned on the WHOLE captured training step (one MI355X).

    python tools/step_tune.py --batches 32,64,128,256 [--model vgg11] [--out table.json]

``tools/conv_tune.py --pairs`` times each layer's pair launch in isolation. In the step the same
launch sits between other kernels, takes the preceding block's BatchNorm-backward sums or its
whole BN backward into its finish, and (one GPU) applies SGD in an unsplit WGRAD epilogue —
round 6 found isolated winners that made the b32 step 3.8 % SLOWER (tools/gpu/ab_variants.sh).
So here: (1) an isolated sweep of every pair candidate (tile x DGRAD split x WGRAD split, plus
the separate launches) keeps the ``--keep`` fastest per layer; (2) coordinate descent over the
layers times each kept candidate inside the real captured step (bench.py's TrainStep:
augment + forward + backward + SGD, ``--reps`` replays, median of ``--trials``), with every other
layer at its current best; a candidate replaces the incumbent only when the step is at least
``--min-gain`` faster. Writes the mode-3 entries of ops/conv_tuning.json (other entries kept).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))

TILES = {0: None, 1: (64, 64), 2: (128, 128), 3: (64, 128), 4: (128, 64), 5: (128, 128)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="vgg11")
    ap.add_argument("--batches", default="32,64,128,256")
    ap.add_argument("--keep", type=int, default=6)
    ap.add_argument("--reps", type=int, default=40)
    ap.add_argument("--trials", type=int, default=3)
    ap.add_argument("--passes", type=int, default=1)
    ap.add_argument("--min-gain", type=float, default=0.003)
    ap.add_argument("--phases", default="pair,fwd",
                    help="pair: the backward-pair entries; fwd: the tap-reuse forward entries")
    ap.add_argument("--merge", default=None)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()

    import torch
    import ddp_amd
    from ddp_amd.data import DeviceLoader, SyntheticCIFAR10
    from ddp_amd.engine import CrossEntropyLoss, TrainStep
    from ddp_amd.models import build
    from ddp_amd.ops.common import TUNING_FILE, native, ptr, workspace
    from ddp_amd.ops.layers import ConvBNActSpec
    from ddp_amd.ops import common
    from ddp_amd.optim import FusedSGD
    from conv_bench import vgg_layers

    n = native()
    dev = torch.device("cuda", 0)
    src = a.merge or TUNING_FILE
    with open(src) as f:
        table = json.load(f)
    # pair entries keyed with the layer's H (different layers share DGRAD GEMM dims)
    entries = {(e["mode"], e["M"], e["N"], e["K"]) + ((e.get("H", 0),) if e["mode"] == 3 else ()): e
               for e in table["entries"]}

    def set_pair(key, tile, sd, sw):
        n.conv_pair_tune_set(key[1], key[2], key[3], key[4] ** 2, tile, sd, sw)

    def isolated(N, C, H, K):
        """Every pair candidate of one layer timed alone: [(us, tile, sd, sw)] sorted."""
        ws = workspace(dev)
        st = torch.cuda.current_stream().cuda_stream
        conv = torch.nn.Conv2d(C, K, 3, 1, 1, bias=False).to(dev)
        conv.weight.data = conv.weight.data.contiguous(memory_format=torch.channels_last)
        spec = ConvBNActSpec(conv, None)
        spec.maybe_pack()
        x = torch.randn(N, H, H, C, device=dev).to(torch.bfloat16)
        dy = torch.randn(N, H, H, K, device=dev).to(torch.bfloat16)
        dx = torch.empty_like(x)
        dw = torch.zeros_like(conv.weight)
        gw = spec.geom(N, H, H, common.weight_krsc(dw))

        def call():
            n.conv_bwd_pair(gw, ptr(dy), ptr(spec.wc), ptr(dx), ptr(x), ptr(dw), ptr(ws),
                            ws.numel(), st)

        def timeit():
            for _ in range(3):
                call()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                call()
            e1.record()
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) * 50.0

        Md, Nd, Kd = N * H * H, C, 9 * K
        Mw, Nw, Kw = K, 9 * C, N * H * H
        out = []
        n.conv_pair_force(0, 0, 0)
        n.conv_pair_mode(0, 0)
        out.append((timeit(), 0, 1, 1))
        n.conv_pair_mode(3, 0)
        kd, kw = (Kd + 63) // 64, (Kw + 63) // 64
        for tile, bmn in TILES.items():
            if bmn is None:
                continue
            for sd in (1, 2, 3, 4, 6, 8, 12, 16):
                if sd > 1 and kd // sd < 2:
                    continue
                for sw in (1, 2, 4, 6, 8, 12, 16, 24, 32, 48, 64):
                    if sw > 1 and kw // sw < 2:
                        continue
                    if (sd * Md * Nd if sd > 1 else 0) + (sw * Mw * Nw if sw > 1 else 0) + 64 > ws.numel():
                        continue
                    n.conv_pair_force(sd, sw, tile)
                    out.append((timeit(), tile, sd, sw))
        n.conv_pair_force(0, 0, 0)
        return sorted(out)

    TR_CANDS = [(bm, bn, sp, ns) for bm in (64, 128) for bn in (64, 128) for sp in (1, 2, 4, 8)
                for ns in (3, 5, 8)]
    tr_entries = {(e["M"], e["K"], e["C"], e["H"]): e for e in table.get("tr_entries", [])}

    def set_tr(key, c):
        n.conv_tr_set(2, key[0], key[1], key[2], key[3], *c)

    def tr_isolated(N, C, H, K):
        """Tap-reuse forward candidates of one layer timed alone (graph replays, us)."""
        from conv_tune_tr import graph_time
        from ddp_amd.ops.common import stream_handle
        ws = workspace(dev)
        conv = torch.nn.Conv2d(C, K, 3, 1, 1).to(dev)
        conv.weight.data = conv.weight.data.contiguous(memory_format=torch.channels_last)
        spec = ConvBNActSpec(conv, None)
        spec.maybe_pack()
        x = torch.randn(N, H, H, C, device=dev).to(torch.bfloat16)
        z = torch.empty(N, H, H, K, device=dev, dtype=torch.bfloat16)
        stats = torch.zeros(16 * 2 * K, device=dev)
        g = spec.geom(N, H, H)

        def tr():
            if not n.conv_fwd_tr(g, ptr(x), ptr(spec.wc), ptr(conv.bias), ptr(z), ptr(stats),
                                 ptr(ws), ws.numel(), stream_handle()):
                raise RuntimeError("not served")
        out = []
        for c in TR_CANDS:
            bm, bn, sp, ns = c
            if K % bn or sp > C // 64:
                continue
            n.conv_tr_set(3, 0, 0, 0, 0, bm, bn, sp, ns)
            try:
                out.append((graph_time(tr), c))
            except RuntimeError:
                pass
            finally:
                n.conv_tr_set(3, 0, 0, 0, 0, 0, 0, 0, 0)
        return sorted(out)

    def step_ms(B, model, opt, loader):
        """Median over trials of the captured step time (ms) with the current table."""
        crit = CrossEntropyLoss()
        res = []
        for _ in range(a.trials):
            st = TrainStep(model, opt, crit, loader)
            st.warmup(2)
            st.capture()
            for _ in range(3):
                st.step()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                st.step()
            e1.record()
            torch.cuda.synchronize()
            res.append(e0.elapsed_time(e1) / a.reps)
            del st
        torch.cuda.empty_cache()
        return sorted(res)[len(res) // 2]

    def tune_fwd(B, layers, model, opt, loader):
        """Coordinate descent over the tap-reuse forward entries (bm = 0: implicit GEMM)."""
        cands, best = {}, {}
        for (N, C, H, K) in layers:
            if H <= 2:  # 2x2 layers run the dense GEMM form (conv_igemm.hip d2x2)
                continue
            key = (N * H * H, K, C, H)
            iso = tr_isolated(N, C, H, K)
            cur = tr_entries.get(key)
            inc = (cur["bm"], cur["bn"], cur["splits"], cur["stages"]) if cur else (0, 0, 0, 0)
            keep = [c for _, c in iso[:a.keep]]
            for c in (inc, (0, 0, 0, 0)):
                if c not in keep:
                    keep.append(c)
            cands[key], best[key] = keep, inc
            set_tr(key, inc)
            print(f"B{B} fwd {C}->{K} {H}x{H}: isolated best {iso[0][0]:.1f} us {iso[0][1]}, "
                  f"incumbent {inc}", flush=True)
        base = t0 = step_ms(B, model, opt, loader)
        for _ in range(a.passes):
            for key, keep in cands.items():
                for c in keep:
                    if c == best[key]:
                        continue
                    set_tr(key, c)
                    ms = step_ms(B, model, opt, loader)
                    if ms < base * (1 - a.min_gain):
                        print(f"  fwd {key}: {best[key]} -> {c}: {base:.4f} -> {ms:.4f} ms",
                              flush=True)
                        best[key], base = c, ms
                    set_tr(key, best[key])
        print(f"B{B} fwd: {t0:.4f} -> {base:.4f} ms", flush=True)
        for key, c in best.items():
            e = tr_entries.get(key, {"M": key[0], "K": key[1], "C": key[2], "H": key[3]})
            e.update(bm=c[0], bn=c[1], splits=c[2], stages=c[3], step_ms=round(base, 4),
                     shape=f"vgg11 N{B} {key[2]}->{key[1]} {key[3]}x{key[3]} (step-tuned)")
            tr_entries[key] = e

    for B in [int(b) for b in a.batches.split(",")]:
        torch.manual_seed(ddp_amd.SEED)
        loader = DeviceLoader(SyntheticCIFAR10(True), B, dev, 1, 0, train=True, cpad=8)
        model = build(a.model).to(dev)
        opt = FusedSGD(model.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
        layers = [(N, C, H, K) for (N, C, H, W, K, R, s, p, Cr) in vgg_layers(B)
                  if C == Cr and s == 1]
        if "fwd" in a.phases:
            tune_fwd(B, layers, model, opt, loader)
        if "pair" not in a.phases:
            continue
        cands = {}
        for (N, C, H, K) in layers:
            key = (3, N * H * H, C, 9 * K, H)
            iso = isolated(N, C, H, K)
            cur = entries.get(key) or entries.get(key[:4] + (0,))
            keep = [(t, sd, sw) for _, t, sd, sw in iso[:a.keep]]
            if cur is not None and (cur["tile"], cur["splits"], cur["stages"]) not in keep:
                keep.append((cur["tile"], cur["splits"], cur["stages"]))
            cands[key] = keep
            print(f"B{B} {C}->{K} {H}x{H}: isolated best {iso[0][0]:.1f} us "
                  f"{iso[0][1:]}, candidates {keep}", flush=True)
        # incumbents: the table's entries (or the isolated best where there is none)
        best = {}
        for key, keep in cands.items():
            cur = entries.get(key) or entries.get(key[:4] + (0,))
            best[key] = (cur["tile"], cur["splits"], cur["stages"]) if cur else keep[0]
            set_pair(key, *best[key])
        base = step_ms(B, model, opt, loader)
        t0 = base
        print(f"B{B}: step with the table's entries {base:.4f} ms", flush=True)
        for _ in range(a.passes):
            for key, keep in cands.items():
                for c in keep:
                    if c == best[key]:
                        continue
                    set_pair(key, *c)
                    ms = step_ms(B, model, opt, loader)
                    if ms < base * (1 - a.min_gain):
                        print(f"  {key[1:]}: {best[key]} -> {c}: {base:.4f} -> {ms:.4f} ms",
                              flush=True)
                        best[key], base = c, ms
                    set_pair(key, *best[key])
        print(f"B{B}: {t0:.4f} -> {base:.4f} ms", flush=True)
        for key, (t, sd, sw) in best.items():
            entries.pop(key[:4] + (0,), None)  # the H-less entry of the same GEMM dims
            entries[key] = {"mode": 3, "M": key[1], "N": key[2], "K": key[3], "H": key[4],
                            "tile": t, "splits": sd, "stages": sw, "step_ms": round(base, 4),
                            "shape": f"vgg11 N{B} {key[2]}->{key[3] // 9} {key[4]}x{key[4]} "
                                     f"pair (step-tuned)"}
        del model, opt, loader
        torch.cuda.empty_cache()
        time.sleep(0.5)
    table["entries"] = list(entries.values())
    table["tr_entries"] = sorted(tr_entries.values(), key=lambda e: (e["H"], e["C"], e["M"]))
    out = a.out or TUNING_FILE
    with open(out, "w") as f:
        json.dump(table, f, indent=1)
    print(f"wrote {len(table['entries'])} entries to {out}")


if __name__ == "__main__":
    main()
