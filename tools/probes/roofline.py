#!/usr/bin/env python3
"""Per-layer roofline of the VGG-11 training GEMMs: ours vs hipBLASLt on the same M/N/K.

For every conv layer and every training GEMM (forward, backward-data, backward-weight):

  ours     our kernels launched exactly as the training step launches them (conv_forward:
           tap-reuse / implicit-GEMM + BN statistics; conv_backward: the DGRAD+WGRAD pair with
           its split-K finish, or WGRAD alone for the input layer), CUDA-event timed
  mm       torch.matmul of the same-shape GEMM with materialised, perfectly streamed operands
           (hipBLASLt, bf16 in / bf16 out): what a vendor GEMM reaches on these dimensions
  peak     2.5 PFLOP/s dense bf16 (MI355X_MICROARCH.md): the per-layer floor flops / peak

GEMM shapes (rows x cols x reduction), N images, HxW, C -> K channels, 3x3 taps:
  fwd    M = N*H*W, N = K, K = 9*C
  dgrad  M = N*H*W, N = C, K = 9*K
  wgrad  M = K,     N = 9*C, K = N*H*W

    python tools/probes/roofline.py --batch 256 [--json out.json]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))

PEAK_TFLOPS = 2500.0
# --trace (round 5): each timed phase is bracketed by marker kernels whose GRID SIZE encodes the
# phase id, so tools/probes/roofline_trace.py can sum the KERNEL durations of a rocprofv3 kernel
# trace per phase. Host-issued launch loops timed with two events (the default) measure the
# dispatch floor on small GEMMs (~18 us for every b32 hipBLASLt cell in round 4), not the GEMM.
TRACE = {"on": False, "phases": [], "marker": None}


def _marker(pid):
    import torch
    from ddp_amd.ops.common import native
    if TRACE["marker"] is None:
        TRACE["marker"] = torch.zeros(4096 * 256 * 16 + 16, dtype=torch.uint8, device="cuda")
    # fill_bytes launches ceil((n / 16 + 1) / 256) workgroups: n = pid * 4096 + 16 -> pid + 1
    native().fill_bytes(TRACE["marker"].data_ptr(), 0, pid * 4096 + 16,
                        torch.cuda.current_stream().cuda_stream)


def timeit(fn, reps=30, label=None):
    import torch
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    if TRACE["on"]:
        pid = len(TRACE["phases"]) + 1
        TRACE["phases"].append({"id": pid, "label": label, "reps": reps})
        _marker(pid)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    if TRACE["on"]:
        _marker(0)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, nargs="+", default=[256])
    ap.add_argument("--json", default=None)
    ap.add_argument("--trace", default=None,
                    help="write the phase list here; run under rocprofv3 --kernel-trace and "
                         "post-process with tools/probes/roofline_trace.py")
    a = ap.parse_args()
    TRACE["on"] = bool(a.trace)
    import torch
    import ddp_amd  # noqa: F401
    from ddp_amd.ops.layers import ConvBNActSpec, conv_forward, conv_backward
    from conv_bench import vgg_layers
    dev = torch.device("cuda", 0)
    rows = []
    for B in a.batch:
        for li, (N, C, H, W, K, R, stride, pad, Cr) in enumerate(vgg_layers(B)):
            conv = torch.nn.Conv2d(Cr, K, R, stride, pad, bias=False).to(dev)
            conv.weight.data = conv.weight.data.contiguous(memory_format=torch.channels_last)
            spec = ConvBNActSpec(conv, None, cin_pad=C if C != Cr else None)
            spec.maybe_pack()
            x = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
            dz = torch.randn(N, H, W, K, device=dev).to(torch.bfloat16)
            dw = torch.zeros_like(conv.weight)
            from ddp_amd.ops.common import stat_replicas
            stats = torch.zeros(stat_replicas() * 2 * K, device=dev)
            M = N * H * W
            gf = 2.0 * M * K * 9 * Cr / 1e9
            shapes = {"fwd": (M, K, 9 * Cr), "dgrad": (M, Cr, 9 * K), "wgrad": (K, 9 * Cr, M)}
            mm = {}
            for name, (m, n, k) in shapes.items():
                A = torch.randn(m, k, device=dev, dtype=torch.bfloat16)
                Bm = torch.randn(k, n, device=dev, dtype=torch.bfloat16)
                mm[name] = timeit(lambda: torch.matmul(A, Bm), label=(B, li, "mm_" + name))
                del A, Bm
            ours = {"fwd": timeit(lambda: conv_forward(spec, x, None, stats), label=(B, li, "ours_fwd"))}
            if li == 0:  # the input layer has no dx
                ours["wgrad"] = timeit(lambda: conv_backward(spec, x, dz, dw, False),
                                       label=(B, li, "ours_bwd"))
                mm_bwd = mm["wgrad"]
                bwd_gf = gf
            else:
                ours["bwd_pair"] = timeit(lambda: conv_backward(spec, x, dz, dw, True),
                                          label=(B, li, "ours_bwd"))
                mm_bwd = mm["dgrad"] + mm["wgrad"]
                bwd_gf = 2 * gf
            ours_bwd = ours.get("bwd_pair", ours.get("wgrad"))
            r = {"batch": B, "layer": li, "shape": f"{Cr}->{K} {H}x{W}", "gflop_fwd": round(gf, 2),
                 "ours_fwd_us": round(ours["fwd"], 2), "mm_fwd_us": round(mm["fwd"], 2),
                 "ours_bwd_us": round(ours_bwd, 2), "mm_dgrad_us": round(mm["dgrad"], 2),
                 "mm_wgrad_us": round(mm["wgrad"], 2),
                 "ours_fwd_tflops": round(gf / ours["fwd"] * 1e3, 1),
                 "mm_fwd_tflops": round(gf / mm["fwd"] * 1e3, 1),
                 "ours_bwd_tflops": round(bwd_gf / ours_bwd * 1e3, 1),
                 "mm_bwd_tflops": round(bwd_gf / mm_bwd * 1e3, 1),
                 "peak_fwd_us": round(gf / PEAK_TFLOPS * 1e3, 2),
                 "peak_bwd_us": round(bwd_gf / PEAK_TFLOPS * 1e3, 2)}
            rows.append(r)
            print(json.dumps(r), flush=True)
        tb = [r for r in rows if r["batch"] == B]
        print(json.dumps({"batch": B, "totals_us": {
            "ours_fwd": round(sum(r["ours_fwd_us"] for r in tb), 1),
            "mm_fwd": round(sum(r["mm_fwd_us"] for r in tb), 1),
            "ours_bwd": round(sum(r["ours_bwd_us"] for r in tb), 1),
            "mm_bwd": round(sum(r["mm_dgrad_us"] + r["mm_wgrad_us"] for r in tb), 1),
            "peak_all": round(sum(r["peak_fwd_us"] + r["peak_bwd_us"] for r in tb), 1)}}),
            flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=1)
    if a.trace:
        with open(a.trace, "w") as f:
            json.dump({"phases": TRACE["phases"], "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
