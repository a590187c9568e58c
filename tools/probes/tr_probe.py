#!/usr/bin/env python3
"""Launch one VGG conv forward a few times through the tap-reuse kernel (forced config) and the
implicit-GEMM kernel, for rocprofv3 --pmc passes (per-dispatch counters, tools/pmc_summary.py).

    python tools/probes/tr_probe.py B C K H bm bn splits stages
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)


def main():
    B, C, K, H, bm, bn, sp, nst = (int(v) for v in sys.argv[1:9])
    import torch
    import ddp_amd
    from ddp_amd.ops.common import ptr, stream_handle, workspace
    from ddp_amd.ops.layers import ConvBNActSpec
    nat = ddp_amd.native()
    dev = torch.device("cuda", 0)
    ws = workspace(dev)
    conv = torch.nn.Conv2d(C, K, 3, 1, 1).to(dev)
    conv.weight.data = conv.weight.data.contiguous(memory_format=torch.channels_last)
    spec = ConvBNActSpec(conv, None)
    spec.maybe_pack()
    x = torch.randn(B, H, H, C, device=dev).to(torch.bfloat16)
    z = torch.empty(B, H, H, K, device=dev, dtype=torch.bfloat16)
    stats = torch.zeros(16 * 2 * K, device=dev)
    g = spec.geom(B, H, H)
    nat.conv_tr_set(3, 0, 0, 0, 0, bm, bn, sp, nst)
    for _ in range(3):
        assert nat.conv_fwd_tr(g, ptr(x), ptr(spec.wc), ptr(conv.bias), ptr(z), ptr(stats),
                               ptr(ws), ws.numel(), stream_handle())
    nat.conv_tr_set(3, 0, 0, 0, 0, 0, 0, 0, 0)
    for _ in range(3):
        nat.conv_fwd(g, ptr(x), ptr(spec.wc), ptr(conv.bias), ptr(z), ptr(stats), ptr(ws),
                     ws.numel(), 0, stream_handle())
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
