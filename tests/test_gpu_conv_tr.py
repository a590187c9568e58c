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
        nat.conv_bn_fuse_rows(128)
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


@pytest.mark.parametrize("N,C,Hz,K,pool,cfg", [
    (8, 128, 16, 256, True, (64, 64, 1)),     # VGG 128 -> pool -> 8x8 conv 256
    (8, 256, 8, 256, False, (128, 64, 1)),    # VGG 256 8x8 -> 8x8 conv (no pool)
    (32, 512, 4, 512, True, (64, 64, 8)),     # 4x4 -> pool -> 2x2, split-K 8
    (16, 256, 8, 512, True, (64, 128, 4)),    # 8x8 -> pool -> 4x4, split-K 4
])
def test_conv_tr_fused_bn_input(native_ext, N, C, Hz, K, pool, cfg):
    """Fused input mode (api.h TrFwdIn): the conv computes its input x = [pool](relu(bn(z)))
    from the preceding block's conv output while loading its patch, writes x (the wgrad operand)
    and the preceding block's coefficient table. Against the separate bn_act_fwd pass + the same
    conv on its output: x and the table bit-identical (same fold order, same formula), z equal."""
    from ddp_amd.ops.common import ptr, stream_handle, workspace
    nat = native_ext
    H = Hz // 2 if pool else Hz
    conv, spec, _, _ = _conv_setup(N, C, H, H, K, 3, 1, 1)
    zin = (torch.randn(N, Hz, Hz, C, device=DEV) * 2 + 0.5).to(torch.bfloat16)
    stats = torch.zeros(16, 2, C, device=DEV)
    zf = zin.float().reshape(-1, C)
    stats[3, 0] = zf.sum(0)  # one replica holds the sums (as the producer's atomics would)
    stats[3, 1] = (zf * zf).sum(0)
    gamma = torch.rand(C, device=DEV) + 0.5
    beta = torch.randn(C, device=DEV) * 0.1
    ws = workspace(torch.device(DEV))
    s = stream_handle()
    g = spec.geom(N, H, H)
    # reference: bn_act_fwd then the conv on its output
    x_ref = torch.empty(N, H, H, C, device=DEV, dtype=torch.bfloat16)
    coef_ref = torch.zeros(6 * C, device=DEV)
    nat.bn_act_fwd(N, Hz, Hz, C, int(pool), 1, 1e-5, ptr(zin), 0, ptr(stats), ptr(gamma),
                   ptr(beta), ptr(x_ref), s, coef=ptr(coef_ref))
    z_ref = torch.empty(N, H, H, K, device=DEV, dtype=torch.bfloat16)
    st_ref = torch.zeros(16 * 2 * K, device=DEV)
    _force(nat, *cfg)
    try:
        assert nat.conv_fwd_tr(g, ptr(x_ref), ptr(spec.wc), ptr(conv.bias), ptr(z_ref),
                               ptr(st_ref), ptr(ws), ws.numel(), s) == 1
        x = torch.full_like(x_ref, float("nan"))
        coef = torch.zeros(6 * C, device=DEV)
        z = torch.empty_like(z_ref)
        st = torch.zeros_like(st_ref)
        fin = (ptr(zin), ptr(stats), ptr(gamma), ptr(beta), 1e-5, 1, int(pool), ptr(coef), ptr(x))
        r = nat.conv_fwd_tr(g, 0, ptr(spec.wc), ptr(conv.bias), ptr(z), ptr(st), ptr(ws),
                            ws.numel(), s, None, fin)
    finally:
        _force(nat, 0, 0, 0)
    torch.cuda.synchronize()
    assert r == 1
    assert torch.equal(x, x_ref), float((x.float() - x_ref.float()).abs().max())
    assert torch.equal(coef[:4 * C], coef_ref[:4 * C])
    assert rel_err(z, z_ref) < 1e-3
    ref = F.conv2d(x_ref.float().permute(0, 3, 1, 2), conv.weight, conv.bias, 1, 1)
    assert rel_err(z.permute(0, 3, 1, 2), ref) < 1e-2


def test_vgg_forward_with_deferred_bn_matches_separate_passes(native_ext):
    """Model level: with the BatchNorm forward of each block deferred into the next block's
    tap-reuse conv (ops/layers.py _defer_bn) the VGG-11 forward and its gradients equal the
    separate-pass forward (same kernels otherwise; only atomics order differs)."""
    import copy
    from ddp_amd.models import VGG11
    from ddp_amd.engine import CrossEntropyLoss
    from ddp_amd.ops import layers
    torch.manual_seed(3)
    base = VGG11().cuda()
    x = torch.randn(32, 3, 32, 32, device=DEV)
    y = torch.randint(0, 10, (32,), device=DEV)
    out = {}
    for fuse in (False, True):
        layers.FUSE_BN_IN = fuse
        try:
            m = copy.deepcopy(base)
            m._plan = None
            loss = CrossEntropyLoss()(m(x), y)
            loss.backward()
            torch.cuda.synchronize()
            ndef = sum(1 for sp in m.fused_plan() if getattr(sp, "last_deferred", False))
            out[fuse] = (float(loss), torch.cat([p.grad.reshape(-1) for p in m.parameters()]))
            if fuse:
                deferred = ndef
            else:
                assert ndef == 0
        finally:
            layers.FUSE_BN_IN = True
    # every block whose next conv the tap-reuse table serves: blocks 1-4 at 32 images (block 0 is
    # the fused input block, conv_l0.hip; blocks 5-6 feed the dense 2x2 GEMMs, conv_igemm.hip
    # d2x2, and block 6's BatchNorm runs inside its own split-K finish)
    assert deferred >= 4, deferred
    assert abs(out[True][0] - out[False][0]) < 1e-3 * abs(out[False][0])
    a, b = out[True][1], out[False][1]
    cos = float(torch.dot(a, b) / (a.norm() * b.norm()))
    assert cos > 0.99, cos
