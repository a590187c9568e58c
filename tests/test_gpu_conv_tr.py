"""Tap-reuse 3x3 forward convolution (csrc/kernels/conv_tr.hip) against fp32 PyTorch and against
the implicit-GEMM kernel on the same bf16 operands.

Reference op: Conv2d(3x3, stride 1, pad 1, bias) of the VGG blocks (/root/reference/part1/
model.py:18-23). Every tile geometry the kernel serves is covered: 16-pixel-wide image bands
(W = 16), whole images of 8x8 / 4x4 / 2x2 (1, 4 and 16 images per tile), 128- and 64-row tiles,
64/128-column tiles, split-K over channel blocks (fp32 slabs + the conv_igemm.hip finish),
and the BatchNorm-fused split-K finish.
"""
import os

import pytest
import torch
import torch.nn.functional as F

from test_gpu_kernels import DEV, _bn_ref, _conv_setup, bf, rel_err  # noqa: F401

pytestmark = pytest.mark.gpu

# N, C, H, K, BM, BN, splits, B-ring stages
TR_CASES = [
    (4, 64, 16, 128, 64, 64, 1, 3),     # W = 16: 4-row bands
    (4, 64, 16, 128, 128, 128, 1, 5),   # 8-row bands, 128x128 tile
    (8, 128, 8, 256, 64, 64, 2, 8),     # one 8x8 image per tile, split-K 2
    (8, 256, 8, 256, 128, 64, 1, 8),    # two images per tile
    (8, 256, 4, 512, 64, 128, 4, 3),    # four 4x4 images per tile, split-K 4
    (16, 512, 4, 512, 128, 64, 1, 5),   # eight 4x4 images
    (32, 512, 2, 512, 64, 64, 8, 5),    # sixteen 2x2 images (pitch-padded patch), split-K 8
    (32, 512, 2, 512, 64, 128, 1, 5),   # 72 k-steps through a 5-deep ring
    (32, 512, 2, 512, 64, 64, 1, 8),    # ... and an 8-deep ring
]


def _force(nat, bm, bn, splits, stages=0):
    nat.conv_tr_set(3, 0, 0, 0, 0, bm, bn, splits, stages)


@pytest.mark.parametrize("case", TR_CASES)
def test_conv_tr_fwd_matches_reference(native_ext, case):
    from ddp_amd.ops.common import ptr, stream_handle, workspace
    nat = native_ext
    N, C, H, K, BM, BN, splits, stages = case
    conv, spec, x, xn = _conv_setup(N, C, H, H, K, 3, 1, 1)
    g = spec.geom(N, H, H)
    ws = workspace(torch.device(DEV))
    s = stream_handle()
    z = torch.full((N, H, H, K), float("nan"), device=DEV, dtype=torch.bfloat16)
    stats = torch.zeros(16 * 2 * K, device=DEV)
    _force(nat, BM, BN, splits, stages)
    try:
        r = nat.conv_fwd_tr(g, ptr(xn), ptr(spec.wc), ptr(conv.bias), ptr(z), ptr(stats),
                            ptr(ws), ws.numel(), s)
    finally:
        _force(nat, 0, 0, 0)
    assert r == 1, "the forced tap-reuse configuration must be served"
    z2 = torch.empty_like(z)
    stats2 = torch.zeros_like(stats)
    nat.conv_fwd(g, ptr(xn), ptr(spec.wc), ptr(conv.bias), ptr(z2), ptr(stats2), ptr(ws),
                 ws.numel(), 0, s)
    torch.cuda.synchronize()
    ref = F.conv2d(x, conv.weight, conv.bias, 1, 1).permute(0, 2, 3, 1)
    assert not torch.isnan(z.float()).any()
    assert rel_err(z, ref) < 1e-2
    # same bf16 operands, fp32 accumulation in a different order: bf16-output level agreement
    assert rel_err(z, z2) < 1e-2
    zf = z.float().reshape(-1, K)
    st = stats.view(16, 2 * K).sum(0)
    assert torch.allclose(st[:K], zf.sum(0), rtol=1e-3, atol=1e-2)
    assert torch.allclose(st[K:], (zf * zf).sum(0), rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("N,C,H,K,pool", [(32, 512, 2, 512, False), (32, 256, 4, 512, True)])
def test_conv_tr_splitk_bn_fused_finish(native_ext, N, C, H, K, pool):
    """Split-K tap-reuse GEMM whose finish also runs the BatchNorm forward (y, coefficient table)
    — the strong-scaling layers' path — against the fp32 reference of conv -> BN -> ReLU (-> pool)."""
    from ddp_amd.ops.common import ptr, stream_handle, workspace
    nat = native_ext
    conv, spec, x, xn = _conv_setup(N, C, H, H, K, 3, 1, 1)
    gamma = torch.rand(K, device=DEV) + 0.5
    beta = torch.randn(K, device=DEV) * 0.1
    Ho = H // 2 if pool else H
    g = spec.geom(N, H, H)
    ws = workspace(torch.device(DEV))
    y = torch.empty(N, Ho, Ho, K, device=DEV, dtype=torch.bfloat16)
    z = torch.empty(N, H, H, K, device=DEV, dtype=torch.bfloat16)
    coef = torch.zeros(6 * K, device=DEV)
    stats = torch.zeros(16 * 2 * K, device=DEV)
    _force(nat, 64, 64, 4)
    nat.conv_bn_fuse_rows(1024)  # every case fused (the shipped limit is 128 rows)
    try:
        r = nat.conv_fwd_tr(g, ptr(xn), ptr(spec.wc), ptr(conv.bias), ptr(z), ptr(stats), ptr(ws),
                            ws.numel(), stream_handle(),
                            (ptr(gamma), ptr(beta), 1e-5, 1, int(pool), ptr(coef), ptr(y), H, H))
    finally:
        _force(nat, 0, 0, 0)
        nat.conv_bn_fuse_rows(int(os.environ.get("DDP_AMD_BN_FUSE_MAX_ROWS", "128")))
    torch.cuda.synchronize()
    assert r == 2, "the split-K GEMM must take the BatchNorm-fused finish"
    zr = F.conv2d(x, conv.weight, conv.bias, 1, 1)
    assert rel_err(z.permute(0, 3, 1, 2), zr) < 1e-2
    ref = _bn_ref(zr, gamma, beta, 1e-5, True, pool, None)
    assert rel_err(y.permute(0, 3, 1, 2), ref) < 1e-2


def test_conv_tr_default_policy_serves_vgg_layers(native_ext):
    """With the shipped policy every VGG-11 3x3 layer after the first is served by the
    tap-reuse kernel at the strong-scaling batches (or explicitly handed back by the table)."""
    from ddp_amd.ops.common import ptr, stream_handle, workspace
    nat = native_ext
    ws = workspace(torch.device(DEV))
    for B in (256, 32):
        for C, K, H in [(64, 128, 16), (128, 256, 8), (256, 256, 8), (256, 512, 4),
                        (512, 512, 4), (512, 512, 2)]:
            conv, spec, x, xn = _conv_setup(B, C, H, H, K, 3, 1, 1)
            z = torch.empty(B, H, H, K, device=DEV, dtype=torch.bfloat16)
            stats = torch.zeros(16 * 2 * K, device=DEV)
            r = nat.conv_fwd_tr(spec.geom(B, H, H), ptr(xn), ptr(spec.wc), ptr(conv.bias), ptr(z),
                                ptr(stats), ptr(ws), ws.numel(), stream_handle())
            if r:
                torch.cuda.synchronize()
                ref = F.conv2d(x, conv.weight, conv.bias, 1, 1).permute(0, 2, 3, 1)
                assert rel_err(z, ref) < 1e-2, (B, C, K, H)
