#!/usr/bin/env python3
"""Sweep the tap-reuse 3x3 forward kernel (csrc/kernels/conv_tr.hip) against the implicit-GEMM
kernel for every VGG-11 3x3 layer at the strong-scaling per-GPU batches, and write the winners
to ops/conv_tuning.json ("tr_entries": (M, K, C, H) -> (bm, bn, splits); bm = 0 keeps the
implicit-GEMM kernel for that layer).

Timing: 20 launches captured in one hipGraph, replayed (device time per launch without host
launch overhead), median of 5 replays, forward op exactly as trained (statistics epilogue,
split-K finish included).

    python tools/conv_tune_tr.py [--batch 256 128 64 32] [--write]
"""
import argparse
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

LAYERS = [(64, 128, 16), (128, 256, 8), (256, 256, 8), (256, 512, 4), (512, 512, 4),
          (512, 512, 2)]
# ResNet-50's stride-1 3x3 convolutions (conv2 of every non-first bottleneck): (C, K, H)
RESNET_LAYERS = [(64, 64, 56), (128, 128, 28), (256, 256, 14), (512, 512, 7)]
CANDS = [(bm, bn, s, n) for bm in (64, 128) for bn in (64, 128) for s in (1, 2, 4, 8)
         for n in (3, 5, 8)]


def graph_time(fn, n=20, reps=5):
    import torch
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1000.0 / n)
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, nargs="+", default=[256, 128, 64, 32])
    ap.add_argument("--write", action="store_true")
    ap.add_argument("--out", default=None,
                    help="write the merged table here instead of over ops/conv_tuning.json")
    ap.add_argument("--model", default="vgg11", choices=["vgg11", "resnet50"],
                    help="layer set of the forward sweep (resnet50: the stride-1 3x3 convs)")
    ap.add_argument("--margin", type=float, default=0.03,
                    help="keep the implicit-GEMM kernel unless tap-reuse is this much faster")
    a = ap.parse_args()
    import torch
    import ddp_amd
    from ddp_amd.ops.common import ptr, stream_handle, workspace, TUNING_FILE
    from ddp_amd.ops.layers import ConvBNActSpec
    nat = ddp_amd.native()
    dev = torch.device("cuda", 0)
    ws = workspace(dev)
    entries = []
    for B in a.batch:
        for C, K, H in (RESNET_LAYERS if a.model == "resnet50" else LAYERS):
            conv = torch.nn.Conv2d(C, K, 3, 1, 1).to(dev)
            conv.weight.data = conv.weight.data.contiguous(memory_format=torch.channels_last)
            spec = ConvBNActSpec(conv, None)
            spec.maybe_pack()
            x = torch.randn(B, H, H, C, device=dev).to(torch.bfloat16)
            z = torch.empty(B, H, H, K, device=dev, dtype=torch.bfloat16)
            stats = torch.zeros(16 * 2 * K, device=dev)
            g = spec.geom(B, H, H)

            def igemm():
                nat.conv_fwd(g, ptr(x), ptr(spec.wc), ptr(conv.bias), ptr(z), ptr(stats), ptr(ws),
                             ws.numel(), 0, stream_handle())

            def tr():
                r = nat.conv_fwd_tr(g, ptr(x), ptr(spec.wc), ptr(conv.bias), ptr(z), ptr(stats),
                                    ptr(ws), ws.numel(), stream_handle())
                if not r:
                    raise RuntimeError("not served")

            base = graph_time(igemm)
            best = (base, (0, 0, 0, 0))
            res = {}
            for bm, bn, s, n in CANDS:
                if K % bn or s > C // 64:
                    continue
                nat.conv_tr_set(3, 0, 0, 0, 0, bm, bn, s, n)
                try:
                    t = graph_time(tr)
                except RuntimeError:
                    continue
                finally:
                    nat.conv_tr_set(3, 0, 0, 0, 0, 0, 0, 0, 0)
                res[f"{bm}x{bn}s{s}n{n}"] = round(t, 2)
                if t < best[0] * (1.0 - a.margin) and t < best[0]:
                    best = (t, (bm, bn, s, n))
            M = B * H * H
            ent = {"M": M, "K": K, "C": C, "H": H, "bm": best[1][0], "bn": best[1][1],
                   "splits": best[1][2], "stages": best[1][3], "us": round(best[0], 2),
                   "igemm_us": round(base, 2),
                   "shape": f"{a.model} N{B} {C}->{K} {H}x{H}"}
            entries.append(ent)
            print(json.dumps(dict(ent, candidates=res)), flush=True)
    if a.write:
        path = os.environ.get("DDP_AMD_CONV_TUNING_FILE", TUNING_FILE)
        with open(path) as f:
            table = json.load(f)
        old = {(e["M"], e["K"], e["C"], e["H"]): e for e in table.get("tr_entries", [])}
        for e in entries:
            old[(e["M"], e["K"], e["C"], e["H"])] = e
        table["tr_entries"] = sorted(old.values(), key=lambda e: (e["H"], e["C"], e["M"]))
        out = a.out or path
        with open(out, "w") as f:
            json.dump(table, f, indent=1)
        print(f"wrote {len(entries)} tap-reuse entries to {out}")


if __name__ == "__main__":
    main()
