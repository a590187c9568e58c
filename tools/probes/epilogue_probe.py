#!/usr/bin/env python3
"""Where does a write-heavy ResNet-50 1x1 conv lose time? (epilogue / statistics / BN passes)

For the layer1 shapes at the bench batch: conv forward with and without the fused BN statistics,
dgrad alone, wgrad alone, the BN-backward reduce + apply passes and a plain bf16 copy of the output
size (the HBM ceiling for the bytes each op must move). CUDA-event timed, back-to-back launches.

    python tools/probes/epilogue_probe.py --batch 256
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)


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
    args = ap.parse_args()
    import torch
    import ddp_amd  # noqa: F401
    from ddp_amd.ops.common import native, ptr, stream_handle
    from ddp_amd.ops.layers import ConvBNActSpec, conv_forward, conv_backward
    dev = torch.device("cuda", 0)
    B = args.batch
    shapes = [(64, 256, 56, 1), (256, 64, 56, 1), (64, 64, 56, 3), (512, 128, 28, 1),
              (128, 512, 28, 1), (1024, 256, 14, 1), (256, 1024, 14, 1)]
    for (C, K, H, R) in shapes:
        conv = torch.nn.Conv2d(C, K, R, 1, R // 2, bias=False).to(dev)
        bn = torch.nn.BatchNorm2d(K).to(dev)
        spec = ConvBNActSpec(conv, bn)
        spec.maybe_pack()
        x = torch.randn(B, H, H, C, device=dev).to(torch.bfloat16)
        dz = torch.randn(B, H, H, K, device=dev).to(torch.bfloat16)
        dw = torch.zeros_like(conv.weight)
        stats = torch.zeros(16 * 2 * K, device=dev)
        out_b = B * H * H * K * 2
        in_b = B * H * H * C * 2
        flops = 2.0 * B * H * H * K * C * R * R
        big = torch.empty(out_b // 2, dtype=torch.bfloat16, device=dev)
        big2 = torch.empty_like(big)
        r = {}
        r["fwd+stats"] = timeit(lambda: conv_forward(spec, x, None, stats))
        r["fwd"] = timeit(lambda: conv_forward(spec, x, None, None))
        r["wgrad"] = timeit(lambda: conv_backward(spec, x, dz, dw, False))
        r["wgrad+dgrad"] = timeit(lambda: conv_backward(spec, x, dz, dw, True))
        r["copy(out)"] = timeit(lambda: big2.copy_(big))
        r["fill(out)"] = timeit(lambda: big2.fill_(1.0))
        if R == 1:  # the same GEMM through hipBLASLt (materialised A, no statistics)
            a2 = x.view(-1, C)
            w2 = torch.randn(C, K, device=dev).to(torch.bfloat16)
            r["torch_mm"] = timeit(lambda: torch.mm(a2, w2))
        native().conv_epi_stage_set(0)
        r["fwd+stats(direct epi)"] = timeit(lambda: conv_forward(spec, x, None, stats))
        native().conv_epi_stage_set(1)
        # BN backward passes over the conv output (reduce -> finalize -> apply, no residual)
        z = conv_forward(spec, x, None, stats)
        y = torch.empty_like(z)
        g, b_ = bn.weight, bn.bias
        N_, P, Q, Kc = z.shape
        native().bn_act_fwd(N_, P, Q, Kc, 0, 1, 1e-5, ptr(z), 0, ptr(stats), ptr(g), ptr(b_), ptr(y),
                            stream_handle(), 0, 0, 0.1, 0, ptr(spec.coef))
        r["bn_fwd"] = timeit(lambda: native().bn_act_fwd(
            N_, P, Q, Kc, 0, 1, 1e-5, ptr(z), 0, ptr(stats), ptr(g), ptr(b_), ptr(y),
            stream_handle(), 0, 0, 0.1, 0, ptr(spec.coef)))
        dzz = torch.empty_like(z)
        gg = torch.zeros(Kc, device=dev)
        gb = torch.zeros(Kc, device=dev)
        sums = torch.zeros(16 * 2 * Kc + 64, device=dev)

        def bwd():
            sums.zero_()
            native().bn_act_bwd(N_, P, Q, Kc, 0, 1, 1e-5, ptr(z), 0, ptr(stats), ptr(g), ptr(b_),
                                ptr(dz), ptr(sums), ptr(dzz), 0, ptr(gg), ptr(gb), 0,
                                stream_handle(), ptr(spec.coef), sums_ready=0)
        r["bn_bwd(zero+reduce+fin+apply)"] = timeit(bwd)
        r["zero"] = timeit(lambda: sums.zero_())
        line = {k: round(v, 1) for k, v in r.items()}
        fl = {k: round(flops / line[k] / 1e6, 0) for k in ("fwd+stats", "fwd")}
        print(f"C{C} K{K} {H}x{H} k{R}: out {out_b / 1e6:.0f} MB in {in_b / 1e6:.0f} MB "
              f"floor(in+out @5TB/s) {(in_b + out_b) / 5e6:.1f} us | {line} | TF/s {fl}", flush=True)


if __name__ == "__main__":
    main()
