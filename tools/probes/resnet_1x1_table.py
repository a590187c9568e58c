#!/usr/bin/env python3
"""ResNet-50 1x1 convolutions: our implicit-GEMM forward vs torch.mm (hipBLASLt) on the same
M/N/K, with and without the BatchNorm statistics epilogue.

Per 1x1 layer (forward GEMM: M = N*P*Q pixels, N = K output channels, K = C input channels):
  ours_stats   conv_forward as trained (bf16 z + per-channel sum / sum-of-squares epilogue)
  ours_plain   conv_forward without statistics (same kernel, no reduction in the epilogue)
  mm           torch.matmul [M, C] x [C, K] bf16 (hipBLASLt), materialised operands

    python tools/probes/resnet_1x1_table.py --batch 256 [--json out.json]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))


def timeit(fn, reps=20):
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
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    import torch
    import ddp_amd  # noqa: F401
    from ddp_amd.ops.layers import ConvBNActSpec, conv_forward
    from conv_bench import resnet_layers
    dev = torch.device("cuda", 0)
    rows = []
    seen = set()
    for (N, C, H, W, K, R, stride, pad, Cr) in resnet_layers(a.batch):
        if R != 1 or stride != 1 or (C, H, K) in seen:
            continue
        seen.add((C, H, K))
        conv = torch.nn.Conv2d(C, K, 1, 1, 0, bias=False).to(dev)
        conv.weight.data = conv.weight.data.contiguous(memory_format=torch.channels_last)
        spec = ConvBNActSpec(conv, None)
        spec.maybe_pack()
        x = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
        stats = torch.zeros(16 * 2 * K, device=dev)
        M = N * H * W
        A = x.view(M, C)
        Bm = torch.randn(C, K, device=dev, dtype=torch.bfloat16)
        gf = 2.0 * M * K * C / 1e9
        r = {"shape": f"{C}->{K} {H}x{W}", "M": M, "N": K, "K": C, "gflop": round(gf, 2),
             "ours_stats_us": timeit(lambda: conv_forward(spec, x, None, stats)),
             "ours_plain_us": timeit(lambda: conv_forward(spec, x, None, None)),
             "mm_us": timeit(lambda: torch.matmul(A, Bm))}
        for k in ("ours_stats", "ours_plain", "mm"):
            r[k + "_tflops"] = round(gf / r[k + "_us"] * 1e3, 1)
            r[k + "_us"] = round(r[k + "_us"], 2)
        r["stats_vs_mm"] = round(r["ours_stats_us"] / r["mm_us"], 2)
        rows.append(r)
        print(json.dumps(r), flush=True)
    print(json.dumps({"totals_us": {k: round(sum(r[k + "_us"] for r in rows), 1)
                                    for k in ("ours_stats", "ours_plain", "mm")}}), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
