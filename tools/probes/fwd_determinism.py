#!/usr/bin/env python3
"""Is the VGG-11 forward run-to-run deterministic, and if not, which block is the first to
differ? Runs the fused block chain twice on one batch (no autograd) and compares each block's
output (deferred BatchNorm outputs are materialised: run with DDP_AMD_FUSE_BN_IN=0 to see
every block), plus the statistics replicas' sums.

    python tools/probes/fwd_determinism.py [--batch 32]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--runs", type=int, default=3)
    a = ap.parse_args()
    import torch
    from ddp_amd.models import VGG11
    from ddp_amd.data import SyntheticCIFAR10, DeviceLoader
    from ddp_amd.ops.layers import conv_bn_act, to_nhwc_input
    from ddp_amd.ops.common import step_scratch
    torch.manual_seed(13)
    m = VGG11().cuda()
    ld = DeviceLoader(SyntheticCIFAR10(True, n=max(256, a.batch)), a.batch, "cuda")
    x, _ = ld.fill(advance=False)
    runs = []
    for _ in range(a.runs):
        outs = []
        with torch.no_grad():
            step_scratch(x.device).zero()
            h = to_nhwc_input(x, 8)
            for spec in m.fused_plan():
                h = conv_bn_act(h, spec)
                torch.cuda.synchronize()
                st = spec.stats.view(16, -1).sum(0)
                outs.append((h.float().clone(), st.clone()))
        runs.append(outs)
    for r in range(1, a.runs):
        for i, ((h0, s0), (h1, s1)) in enumerate(zip(runs[0], runs[r])):
            dh = float((h1 - h0).norm() / (h0.norm() + 1e-30))
            ds = float((s1 - s0).norm() / (s0.norm() + 1e-30))
            neq = int((h1 != h0).sum())
            print(f"run {r} block {i}: out rel diff {dh:.3e} ({neq} of {h0.numel()} differ), "
                  f"stats rel diff {ds:.3e}")


if __name__ == "__main__":
    main()
