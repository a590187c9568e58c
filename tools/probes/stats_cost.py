#!/usr/bin/env python3
"""How much do the fused BatchNorm-statistics atomics cost the conv forward kernels?
Times each VGG-11 b256 forward conv with and without the stats pointer."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))


def main():
    import torch
    import ddp_amd  # noqa: F401
    from ddp_amd.ops.common import native, ptr, workspace
    from ddp_amd.ops.layers import ConvBNActSpec
    from conv_bench import vgg_layers
    n = native()
    dev = torch.device("cuda", 0)
    ws = workspace(dev)
    st = torch.cuda.current_stream().cuda_stream

    def timeit(fn, reps=50):
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

    for (N, C, H, W, K, R, stride, pad, Cr) in vgg_layers(256):
        conv = torch.nn.Conv2d(Cr, K, R, stride, pad).to(dev)
        spec = ConvBNActSpec(conv, None, cin_pad=C if C != Cr else None)
        spec.maybe_pack()
        x = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
        z = torch.empty(N, H, W, K, device=dev, dtype=torch.bfloat16)
        stats = torch.zeros(16 * 2 * K, device=dev)
        g = spec.geom(N, H, W)
        if C == 8:
            f = lambda s: n.conv_fwd_smallk(g, ptr(x), ptr(spec.wc), ptr(conv.bias), ptr(z), s, st)  # noqa
        else:
            f = lambda s: n.conv_fwd(g, ptr(x), ptr(spec.wc), ptr(conv.bias), ptr(z), s, ptr(ws),  # noqa
                                     ws.numel(), 0, st)
        a = timeit(lambda: f(ptr(stats)))
        b = timeit(lambda: f(0))
        print(f"N{N} {Cr}->{K} {H}x{W}: with stats {a:6.1f} us, without {b:6.1f} us", flush=True)


if __name__ == "__main__":
    main()
