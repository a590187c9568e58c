"""Numerics of every gfx950 kernel against a plain PyTorch fp32 reference of the same op.

Inputs are bf16-representable (the kernels consume bf16 activations/weights), references run in
fp32 (or fp64) on the same values; tolerances are bf16-output level.
"""
import os

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


def bf(t):
    return t.to(torch.bfloat16).float()


def rel_err(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-12))


CONV_CASES = [
    # N, Cin, H, W, K, R, stride, pad
    (4, 64, 16, 16, 128, 3, 1, 1),
    (2, 8, 32, 32, 64, 3, 1, 1),     # VGG layer 0 (padded channels)
    (8, 512, 2, 2, 512, 3, 1, 1),    # deep tiny-spatial layer (split-K)
    (4, 64, 15, 15, 32, 3, 2, 1),    # stride 2, odd size
    (2, 128, 14, 14, 256, 1, 1, 0),  # 1x1
    (2, 64, 14, 14, 128, 1, 2, 0),   # 1x1 stride 2
    (2, 8, 32, 32, 64, 7, 2, 3),     # 7x7 stem-like
    (3, 8, 40, 40, 64, 7, 2, 3),     # stem, partial last pixel-tile group
    (128, 8, 224, 224, 64, 7, 2, 3),  # stem: full grid, waves walk several pixel-tile groups
]


def _conv_setup(N, Cin, H, W, K, R, stride, pad, Creal=None):
    from ddp_amd.ops.layers import ConvBNActSpec
    Creal = Creal or Cin
    conv = torch.nn.Conv2d(Creal, K, R, stride, pad, bias=True).to(DEV)
    with torch.no_grad():
        conv.weight.copy_(bf(conv.weight))
        conv.bias.copy_(torch.randn_like(conv.bias) * 0.1)
    spec = ConvBNActSpec(conv, None, cin_pad=Cin)
    spec.maybe_pack()
    x = bf(torch.randn(N, Creal, H, W, device=DEV))
    x_nhwc = torch.zeros(N, H, W, Cin, device=DEV, dtype=torch.bfloat16)
    x_nhwc[..., :Creal] = x.permute(0, 2, 3, 1).to(torch.bfloat16)
    return conv, spec, x, x_nhwc


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_fwd_stats(native_ext, case):
    from ddp_amd.ops.layers import conv_forward
    N, Cin, H, W, K, R, stride, pad = case
    Creal = 3 if Cin == 8 else Cin
    conv, spec, x, xn = _conv_setup(N, Cin, H, W, K, R, stride, pad, Creal)
    stats = torch.zeros(16 * 2 * K, device=DEV)
    z = conv_forward(spec, xn, conv.bias, stats)
    stats = stats.view(16, 2 * K).sum(0)
    ref = F.conv2d(x, conv.weight, conv.bias, stride, pad).permute(0, 2, 3, 1)
    assert z.shape == ref.shape
    assert rel_err(z, ref) < 1e-2
    zf = z.float().reshape(-1, K)
    assert torch.allclose(stats[:K], zf.sum(0), rtol=1e-3, atol=1e-2)
    assert torch.allclose(stats[K:], (zf * zf).sum(0), rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("layout", ["kcrs", "krsc", "krsc_deep"])
@pytest.mark.parametrize("case", [c for c in CONV_CASES if c[1] != 8])
def test_conv_dgrad(native_ext, case, layout):
    """dgrad + wgrad; the weight gradient in the standard [K][C][R][S] layout and the GPU arena's
    [K][R][S][C] layout (also with the deepest LDS ring)."""
    from ddp_amd.ops.layers import conv_backward
    N, Cin, H, W, K, R, stride, pad = case
    conv, spec, x, xn = _conv_setup(N, Cin, H, W, K, R, stride, pad)
    P = (H + 2 * pad - R) // stride + 1
    dz = bf(torch.randn(N, K, P, P, device=DEV))
    dzn = dz.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16)
    fmt = torch.contiguous_format if layout == "kcrs" else torch.channels_last
    dw = torch.zeros_like(conv.weight, memory_format=fmt)
    native_ext.conv_options(4 if layout == "krsc_deep" else (3 if layout == "krsc" else 2))
    try:
        dx = conv_backward(spec, xn, dzn, dw, True)
        torch.cuda.synchronize()
    finally:
        from ddp_amd.ops.common import CONV_STAGES
        native_ext.conv_options(CONV_STAGES)
    xr = x.clone().requires_grad_(True)
    wr = conv.weight.detach().clone().requires_grad_(True)
    out = F.conv2d(xr, wr, None, stride, pad)
    out.backward(dz)
    assert rel_err(dx.permute(0, 3, 1, 2), xr.grad) < 1e-2
    assert rel_err(dw, wr.grad) < 1e-2


@pytest.mark.parametrize("mode", [0, 1, 2, 3])
@pytest.mark.parametrize("case", [(32, 512, 2, 2, 512, 3, 1, 1), (32, 256, 4, 4, 512, 3, 1, 1),
                                  (32, 64, 16, 16, 128, 3, 1, 1), (2, 128, 14, 14, 256, 1, 1, 0),
                                  (4, 64, 15, 15, 32, 3, 2, 1)])
def test_conv_bwd_pair(native_ext, case, mode):
    """One layer's wgrad + dgrad as ONE grouped launch (+ one grouped split-K finish):
    ddp_conv_bwd_pair, policy 0 = two launches, 1 = paired when both pick 64x64, 2 = always
    paired (stride 1), 3 = 1 or small enough; all must match the fp32 reference."""
    from ddp_amd.ops.layers import conv_backward
    N, Cin, H, W, K, R, stride, pad = case
    conv, spec, x, xn = _conv_setup(N, Cin, H, W, K, R, stride, pad)
    P = (H + 2 * pad - R) // stride + 1
    dz = bf(torch.randn(N, K, P, P, device=DEV))
    dzn = dz.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16)
    dw = torch.zeros_like(conv.weight, memory_format=torch.channels_last)
    native_ext.conv_pair_mode(mode)
    try:
        dx = conv_backward(spec, xn, dzn, dw, True)
        torch.cuda.synchronize()
    finally:
        native_ext.conv_pair_mode(3)
    xr = x.clone().requires_grad_(True)
    wr = conv.weight.detach().clone().requires_grad_(True)
    F.conv2d(xr, wr, None, stride, pad).backward(dz)
    assert rel_err(dx.permute(0, 3, 1, 2), xr.grad) < 1e-2
    assert rel_err(dw, wr.grad) < 1e-2


@pytest.mark.parametrize("tile", [1, 2, 3, 4, 5])
@pytest.mark.parametrize("sd,sw", [(1, 1), (1, 8), (3, 4), (6, 1), (4, 24)])
@pytest.mark.parametrize("case", [(32, 512, 2, 2, 512, 3, 1, 1), (32, 64, 16, 16, 128, 3, 1, 1),
                                  (32, 256, 4, 4, 512, 3, 1, 1), (16, 128, 8, 8, 256, 3, 1, 1)])
def test_conv_bwd_pair_forced_splits(native_ext, case, sd, sw, tile):
    """The measured pair entries (table mode 3, tools/conv_tune.py --pairs) fix the pair tile
    (1 = 64x64, 2 = 128x128, 3 = 64x128, 4 = 128x64) and the DGRAD / WGRAD split-K factors of the
    grouped launch: every (tile, sd, sw) the sweep may pick matches fp32."""
    from ddp_amd.ops.layers import conv_backward
    N, Cin, H, W, K, R, stride, pad = case
    conv, spec, x, xn = _conv_setup(N, Cin, H, W, K, R, stride, pad)
    dz = bf(torch.randn(N, K, H, W, device=DEV))
    dzn = dz.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16)
    dw = torch.zeros_like(conv.weight, memory_format=torch.channels_last)
    native_ext.conv_pair_force(sd, sw, tile)
    try:
        dx = conv_backward(spec, xn, dzn, dw, True)
        torch.cuda.synchronize()
    finally:
        native_ext.conv_pair_force(0, 0, 0)
    xr = x.clone().requires_grad_(True)
    wr = conv.weight.detach().clone().requires_grad_(True)
    F.conv2d(xr, wr, None, stride, pad).backward(dz)
    assert rel_err(dx.permute(0, 3, 1, 2), xr.grad) < 1e-2
    assert rel_err(dw, wr.grad) < 1e-2


@pytest.mark.parametrize("pm", [1, 2, 0])
@pytest.mark.parametrize("tile,sd,sw", [(0, 1, 1), (1, 1, 1), (1, 2, 4), (2, 3, 2), (2, 1, 6),
                                        (3, 2, 3), (4, 1, 8), (5, 1, 4)])
@pytest.mark.parametrize("case", [(64, 512, 2, 2, 512), (64, 256, 4, 4, 512), (128, 512, 4, 4, 512),
                                  (64, 256, 8, 8, 256), (128, 128, 8, 8, 256), (64, 64, 16, 16, 128),
                                  (64, 64, 14, 14, 64)])
def test_conv_wgrad_pixel_major(native_ext, case, tile, sd, sw, pm):
    """Pixel-major WGRAD reduction (conv_igemm.hip ConvArgs::pixmajor: (pixel, 64 images)
    k-steps, the taps' padding k-steps skipped, scalar-offset gathers) on the 2x2 / 4x4 / 8x8
    layers at 64 / 128 images, as the pair's WGRAD half (tile 1..5, forced splits) and as the
    separate launch (tile 0), against fp32 PyTorch — pm = 2 also on the 16x16 / 14x14 images
    (the tap's valid pixels walked as a rectangle), pm = 0 (pixel order) the same."""
    from ddp_amd.ops.layers import conv_backward
    N, Cin, H, W, K = case
    conv, spec, x, xn = _conv_setup(N, Cin, H, W, K, 3, 1, 1)
    dz = bf(torch.randn(N, K, H, W, device=DEV))
    dzn = dz.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16)
    dw = torch.zeros_like(conv.weight, memory_format=torch.channels_last)
    native_ext.conv_wgrad_pm_set(pm)
    if tile == 0:
        native_ext.conv_pair_mode(0)
    else:
        native_ext.conv_pair_force(sd, sw, tile)
    try:
        dx = conv_backward(spec, xn, dzn, dw, True)
        torch.cuda.synchronize()
    finally:
        native_ext.conv_wgrad_pm_set(1)
        native_ext.conv_pair_force(0, 0, 0)
        native_ext.conv_pair_mode(3)
    xr = x.clone().requires_grad_(True)
    wr = conv.weight.detach().clone().requires_grad_(True)
    F.conv2d(xr, wr, None, 1, 1).backward(dz)
    assert rel_err(dx.permute(0, 3, 1, 2), xr.grad) < 1e-2
    assert rel_err(dw, wr.grad) < 1e-2


@pytest.mark.parametrize("rows_pm", [1, 2, 0])
@pytest.mark.parametrize("tile", [0, 1, 2, 3, 4, 5, 6, 7])
@pytest.mark.parametrize("splits", [0, 3])
@pytest.mark.parametrize("case", [(128, 256, 4, 4, 512), (256, 128, 8, 8, 256),
                                  (128, 512, 2, 2, 512), (64, 512, 4, 4, 256),
                                  (64, 64, 16, 16, 128), (64, 64, 14, 14, 64)])
def test_conv_rows_pixel_major(native_ext, case, splits, tile, rows_pm):
    """Pixel-major FWD / DGRAD rows (conv_igemm.hip ConvArgs::pixmajor: a row tile = one pixel of
    BM images, the padding taps' k-steps skipped, NHWC epilogue / slab rows) on every forced tile
    (pixel-major only where BM divides the batch), unsplit and split 3 ways (slabs + finish),
    the BN statistics of the rounded z included — against fp32 PyTorch; rows_pm = 2 also takes
    the images above 64 pixels (16x16, 14x14), rows_pm = 0 none."""
    from ddp_amd.ops.common import ptr, stream_handle, workspace
    N, Cin, H, W, K = case
    conv, spec, x, xn = _conv_setup(N, Cin, H, W, K, 3, 1, 1)
    ws = workspace(xn.device)
    g = spec.geom(N, H, W)
    z = torch.empty(N, H, W, K, dtype=torch.bfloat16, device=DEV)
    stats = torch.zeros(16 * 2 * K, device=DEV)
    dz = bf(torch.randn(N, K, H, W, device=DEV))
    dzn = dz.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16)
    dx = torch.empty_like(xn)
    native_ext.conv_rows_pm_set(rows_pm)
    native_ext.conv_force_tile(tile + 1, 0)
    native_ext.conv_dense2x2_set(0)  # (2x2: the implicit GEMM, so the rows path is exercised)
    try:
        native_ext.conv_fwd(g, ptr(xn), ptr(spec.wc), ptr(conv.bias), ptr(z), ptr(stats), ptr(ws),
                            ws.numel(), splits, stream_handle())
        native_ext.conv_dgrad(g, ptr(dzn), ptr(spec.wc), ptr(dx), ptr(ws), ws.numel(), splits,
                              stream_handle())
        torch.cuda.synchronize()
    finally:
        native_ext.conv_rows_pm_set(1)
        native_ext.conv_force_tile(0, 0)
        native_ext.conv_dense2x2_set(1)
    ref = F.conv2d(x, conv.weight, conv.bias, 1, 1).permute(0, 2, 3, 1)
    assert rel_err(z, ref) < 1e-2
    zf = z.float().reshape(-1, K)
    st = stats.view(16, 2 * K).sum(0)
    assert torch.allclose(st[:K], zf.sum(0), rtol=1e-3, atol=1e-2)
    assert torch.allclose(st[K:], (zf * zf).sum(0), rtol=1e-3, atol=1e-2)
    xr = x.clone().requires_grad_(True)
    F.conv2d(xr, conv.weight.detach(), None, 1, 1).backward(dz)
    assert rel_err(dx.permute(0, 3, 1, 2), xr.grad) < 1e-2


@pytest.mark.parametrize("fmt", [torch.contiguous_format, torch.channels_last])
def test_conv_wgrad_padded_layer0(native_ext, fmt):
    from ddp_amd.ops.layers import conv_backward
    conv, spec, x, xn = _conv_setup(4, 8, 32, 32, 64, 3, 1, 1, Creal=3)
    dz = bf(torch.randn(4, 64, 32, 32, device=DEV))
    dw = torch.zeros_like(conv.weight, memory_format=fmt)
    conv_backward(spec, xn, dz.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16), dw, False)
    wr = conv.weight.detach().clone().requires_grad_(True)
    F.conv2d(x, wr, None, 1, 1).backward(dz)
    assert rel_err(dw, wr.grad) < 1e-2


def _bn_ref(z, gamma, beta, eps, relu, pool, res=None):
    # z: NCHW fp32 (bf16-valued)
    y = F.batch_norm(z, None, None, gamma, beta, training=True, eps=eps)
    if res is not None:
        y = y + res
    if relu:
        y = F.relu(y)
    if pool:
        y = F.max_pool2d(y, 2, 2)
    return y


@pytest.mark.parametrize("N,C,H,pool,res", [(8, 64, 8, True, False), (8, 128, 4, False, False),
                                            (8, 512, 2, True, False), (8, 256, 8, False, True),
                                            (8, 2048, 2, False, True), (16, 128, 16, True, False),
                                            (32, 256, 8, False, False), (16, 256, 8, False, True),
                                            (32, 64, 8, True, False)])
@pytest.mark.parametrize("mode", ["split", "local", "mask", "mask-local"])
def test_bn_act_fwd_bwd(native_ext, N, C, H, pool, res, mode):
    """split: reduce -> finalize -> apply launches; local: one block per 8 channels does the
    whole backward in one launch (bn_act_bwd_local_kernel; the shapes cover 1-8 items per
    thread, pooled, plain and residual). mask: residual blocks whose forward stores the ReLU
    mask bits (BnArgs::mask) and whose backward reads them instead of the residual — must be
    BITWISE equal to the residual-reading backward."""
    from ddp_amd.ops.common import ptr, stream_handle
    nat = native_ext
    if mode.startswith("mask") and not res:
        pytest.skip("the ReLU mask serves residual blocks only")
    nat.bn_bwd_local_set(64 if mode.endswith("local") else 0)  # local: any shape it can hold
    try:
        _bn_case(nat, N, C, H, pool, res, mode, ptr, stream_handle)
        if mode.endswith("local"):
            assert nat.bn_bwd_local_ok(N, H, H, C, int(pool))
    finally:
        nat.bn_bwd_local_set(8)  # the shipped limit (bn_act.hip kLocalMaxLoads)


@pytest.mark.parametrize("N,C,H,pool,res", [(128, 256, 28, False, True), (128, 128, 56, True, False)])
def test_bn_act_big_grid_fold(native_ext, N, C, H, pool, res):
    """Layers big enough for the capped-grid FOLD launches (bn_act.hip: the forward apply and the
    backward apply walk their item blocks with a grid stride and fold the finalize once per
    block) against the fp32 PyTorch reference."""
    from ddp_amd.ops.common import ptr, stream_handle
    _bn_case(native_ext, N, C, H, pool, res, "split", ptr, stream_handle)


def _bn_case(nat, N, C, H, pool, res, mode, ptr, stream_handle):
    z = bf(torch.randn(N, C, H, H, device=DEV) * 2 + 0.5)
    r = bf(torch.randn(N, C, H, H, device=DEV)) if res else None
    gamma = torch.rand(C, device=DEV) + 0.5
    beta = torch.randn(C, device=DEV) * 0.1
    zn = z.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16)
    rn = r.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16) if res else None
    zf = zn.float().reshape(-1, C)
    stats = torch.zeros(16, 2 * C, device=DEV)  # 16 contention-spreading replicas
    stats[3] = torch.cat([zf.sum(0), (zf * zf).sum(0)])
    Ho = H // 2 if pool else H
    out = torch.empty(N, Ho, Ho, C, device=DEV, dtype=torch.bfloat16)
    s = stream_handle()
    coef = torch.empty(6 * C, device=DEV)
    use_mask = mode.startswith("mask")
    mask = torch.full((N, H, H, C // 8), 0xA5, dtype=torch.uint8, device=DEV) if use_mask else None
    nat.bn_act_fwd(N, H, H, C, int(pool), 1, 1e-5, ptr(zn), ptr(rn), ptr(stats), ptr(gamma),
                   ptr(beta), ptr(out), s, coef=ptr(coef), mask=ptr(mask))
    zr = z.clone().requires_grad_(True)
    gr = gamma.clone().requires_grad_(True)
    br = beta.clone().requires_grad_(True)
    rr = r.clone().requires_grad_(True) if res else None
    ref = _bn_ref(zr, gr, br, 1e-5, True, pool, rr)
    assert rel_err(out.permute(0, 3, 1, 2), ref) < 1e-2
    dout = bf(torch.randn_like(ref))
    ref.backward(dout)
    doutn = dout.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16)
    sums = torch.zeros(16 * 2 * C, device=DEV)  # 16 replicas of [2][C]
    dz = torch.empty_like(zn)
    dres = torch.empty_like(zn) if res else None
    dg = torch.zeros(C, device=DEV)
    db = torch.zeros(C, device=DEV)
    dbias = torch.zeros(C, device=DEV)
    nat.bn_act_bwd(N, H, H, C, int(pool), 1, 1e-5, ptr(zn), ptr(rn), ptr(stats), ptr(gamma),
                   ptr(beta), ptr(doutn), ptr(sums), ptr(dz), ptr(dres), ptr(dg), ptr(db),
                   ptr(dbias), s, ptr(coef))
    torch.cuda.synchronize()
    if use_mask:
        # the mask bits are exactly the pre-ReLU sign test of the forward
        y_pre = (zn.float() * coef[:C] + coef[C:2 * C] + rn.float())
        bits = (y_pre > 0).reshape(N, H, H, C // 8, 8).to(torch.int32)
        want = (bits << torch.arange(8, device=DEV, dtype=torch.int32)).sum(-1)
        assert torch.equal(mask.to(torch.int32), want)
        # the mask-reading backward (residual pointer null) is bitwise the residual-reading one
        sums_m = torch.zeros_like(sums)
        dz_m, dres_m = torch.empty_like(zn), torch.empty_like(zn)
        dg_m, db_m = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
        nat.bn_act_bwd(N, H, H, C, int(pool), 1, 1e-5, ptr(zn), 0, ptr(stats), ptr(gamma),
                       ptr(beta), ptr(doutn), ptr(sums_m), ptr(dz_m), ptr(dres_m), ptr(dg_m),
                       ptr(db_m), 0, s, ptr(coef), mask=ptr(mask))
        torch.cuda.synchronize()
        assert torch.equal(dres_m, dres)
        if mode.endswith("local"):  # in-block sums: no atomics, the whole backward is bitwise
            assert torch.equal(dz_m, dz)
        else:  # replica sums through float atomics: equal up to their summation order
            assert rel_err(dz_m.float(), dz.float()) < 1e-3
        assert torch.allclose(dg_m, dg, rtol=1e-5, atol=1e-5)
        assert torch.allclose(db_m, db, rtol=1e-5, atol=1e-5)
    assert rel_err(dz.permute(0, 3, 1, 2), zr.grad) < 2e-2
    assert rel_err(dg, gr.grad) < 1e-2
    assert rel_err(db, br.grad) < 1e-2
    # conv-bias gradient through train-mode BN is identically zero (left untouched)
    assert torch.allclose(dbias, zr.grad.sum((0, 2, 3)), atol=5e-2)
    if res:
        assert rel_err(dres.permute(0, 3, 1, 2), rr.grad) < 1e-2


@pytest.mark.parametrize("N,C,H", [(8, 256, 8), (64, 256, 28), (8, 2048, 4), (16, 1024, 7)])
def test_bn_act_shortcut_bn(native_ext, N, C, H):
    """Residual block with the projection shortcut's BatchNorm folded in (bn_act.hip RBN):
    y = relu(bn(z) + bn_r(zr)) from ONE finalize + apply, and the backward's reduce (three sums,
    S1 shared) + dual finalize + apply write dz AND the shortcut's dz, both BNs' gamma / beta
    gradients, against fp32 PyTorch. (64, 256, 28) takes the 4-items-per-thread forward and
    the capped-grid (grid-stride) reduce."""
    from ddp_amd.ops.common import ptr, stream_handle
    nat = native_ext
    s = stream_handle()
    eps = 1e-5
    z = bf(torch.randn(N, C, H, H, device=DEV) * 2 + 0.5)
    zr = bf(torch.randn(N, C, H, H, device=DEV) * 0.7 - 0.3)
    g, b = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV) * 0.1
    gr, br = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV) * 0.1
    zn = z.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16)
    zrn = zr.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16)

    def stats_of(t):
        tf = t.float().reshape(-1, C)
        st = torch.zeros(16, 2 * C, device=DEV)
        st[5] = torch.cat([tf.sum(0), (tf * tf).sum(0)])
        return st

    st, str_ = stats_of(zn), stats_of(zrn)
    coef, rcoef = torch.empty(6 * C, device=DEV), torch.empty(6 * C, device=DEV)
    rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    rrm, rrv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    out = torch.empty(N, H, H, C, device=DEV, dtype=torch.bfloat16)
    mask = torch.full((N, H, H, C // 8), 0xA5, dtype=torch.uint8, device=DEV)
    nat.bn_act_fwd(N, H, H, C, 0, 1, eps, ptr(zn), ptr(zrn), ptr(st), ptr(g), ptr(b), ptr(out), s,
                   ptr(rm), ptr(rv), 0.1, 0, ptr(coef), mask=ptr(mask), rstats=ptr(str_),
                   rgamma=ptr(gr), rbeta=ptr(br), rcoef=ptr(rcoef), rrunning_mean=ptr(rrm),
                   rrunning_var=ptr(rrv), reps=eps, rmomentum=0.1)
    zq = z.clone().requires_grad_(True)
    zrq = zr.clone().requires_grad_(True)
    gq, bq = g.clone().requires_grad_(True), b.clone().requires_grad_(True)
    grq, brq = gr.clone().requires_grad_(True), br.clone().requires_grad_(True)
    rm_ref, rv_ref = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    rrm_ref, rrv_ref = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    ref = F.relu(F.batch_norm(zq, rm_ref, rv_ref, gq, bq, training=True, eps=eps)
                 + F.batch_norm(zrq, rrm_ref, rrv_ref, grq, brq, training=True, eps=eps))
    torch.cuda.synchronize()
    assert rel_err(out.permute(0, 3, 1, 2), ref) < 1e-2
    for mine, want in ((rm, rm_ref), (rv, rv_ref), (rrm, rrm_ref), (rrv, rrv_ref)):
        assert torch.allclose(mine, want, rtol=1e-4, atol=1e-5)
    # the mask bits are the pre-ReLU sign test of the forward's own arithmetic
    y_pre = (zn.float() * coef[:C] + coef[C:2 * C]) + (zrn.float() * rcoef[:C] + rcoef[C:2 * C])
    bits = (y_pre > 0).reshape(N, H, H, C // 8, 8).to(torch.int32)
    want = (bits << torch.arange(8, device=DEV, dtype=torch.int32)).sum(-1)
    assert (mask.to(torch.int32) != want).float().mean() < 1e-4  # (fma rounding at y == 0)
    dout = bf(torch.randn_like(ref))
    ref.backward(dout)
    doutn = dout.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16)
    sums = torch.zeros(16 * 2 * C + 64, device=DEV)
    rsums = torch.zeros(16 * 2 * C + 64, device=DEV)
    dz, dzr = torch.empty_like(zn), torch.empty_like(zn)
    dg, db = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
    dgr, dbr = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
    nat.bn_act_bwd(N, H, H, C, 0, 1, eps, ptr(zn), ptr(zrn), ptr(st), ptr(g), ptr(b),
                   ptr(doutn), ptr(sums), ptr(dz), 0, ptr(dg), ptr(db), 0, s, ptr(coef),
                   mask=ptr(mask), rcoef=ptr(rcoef), rsums=ptr(rsums), rdz=ptr(dzr),
                   rdgamma=ptr(dgr), rdbeta=ptr(dbr))
    torch.cuda.synchronize()
    assert rel_err(dz.permute(0, 3, 1, 2), zq.grad) < 2e-2
    assert rel_err(dzr.permute(0, 3, 1, 2), zrq.grad) < 2e-2
    assert rel_err(dg, gq.grad) < 1e-2 and rel_err(db, bq.grad) < 1e-2
    assert rel_err(dgr, grq.grad) < 1e-2 and rel_err(dbr, brq.grad) < 1e-2
    # eval: both tables from the running statistics
    rm2, rv2 = torch.randn(C, device=DEV) * 0.1, torch.rand(C, device=DEV) + 0.5
    rrm2, rrv2 = torch.randn(C, device=DEV) * 0.1, torch.rand(C, device=DEV) + 0.5
    nat.bn_act_fwd(N, H, H, C, 0, 1, eps, ptr(zn), ptr(zrn), ptr(st), ptr(g), ptr(b), ptr(out), s,
                   ptr(rm2), ptr(rv2), 0.1, 1, ptr(coef), rstats=ptr(str_), rgamma=ptr(gr),
                   rbeta=ptr(br), rcoef=ptr(rcoef), rrunning_mean=ptr(rrm2),
                   rrunning_var=ptr(rrv2), reps=eps, rmomentum=0.1)
    torch.cuda.synchronize()
    ev = F.relu(F.batch_norm(z, rm2, rv2, g, b, training=False, eps=eps)
                + F.batch_norm(zr, rrm2, rrv2, gr, br, training=False, eps=eps))
    assert rel_err(out.permute(0, 3, 1, 2), ev) < 1e-2


def test_linear_ce(native_ext):
    from ddp_amd.ops.layers import linear_small, cross_entropy
    B, Fi, J = 64, 512, 10
    lin = torch.nn.Linear(Fi, J).to(DEV)
    x = bf(torch.randn(B, Fi, device=DEV))
    y = torch.randint(0, J, (B,), device=DEV)
    lin.weight.grad = torch.zeros_like(lin.weight)
    lin.bias.grad = torch.zeros_like(lin.bias)
    xb = x.to(torch.bfloat16).requires_grad_(True)
    logits = linear_small(xb, lin)
    loss = cross_entropy(logits, y)
    loss.backward()
    xr = x.clone().requires_grad_(True)
    wr = lin.weight.detach().clone().requires_grad_(True)
    brr = lin.bias.detach().clone().requires_grad_(True)
    lr_ = F.linear(xr, wr, brr)
    lref = F.cross_entropy(lr_, y)
    lref.backward()
    assert rel_err(logits, lr_) < 1e-4
    assert abs(float(loss) - float(lref)) < 1e-4
    assert rel_err(xb.grad, xr.grad) < 1e-2
    assert rel_err(lin.weight.grad, wr.grad) < 1e-4
    assert rel_err(lin.bias.grad, brr.grad) < 1e-4


def test_softmax_ce_bf16_1000(native_ext):
    from ddp_amd.ops.common import ptr, stream_handle
    B, J = 32, 1000
    logits = bf(torch.randn(B, J, device=DEV) * 3)
    y = torch.randint(0, J, (B,), device=DEV)
    loss = torch.zeros((), device=DEV)
    correct = torch.zeros((), dtype=torch.int32, device=DEV)
    dl = torch.empty(B, J, device=DEV, dtype=torch.bfloat16)
    native_ext.softmax_ce(ptr(logits.to(torch.bfloat16)), 1, ptr(y), B, J, ptr(loss), ptr(correct),
                          ptr(dl), 1, stream_handle())
    torch.cuda.synchronize()
    lr_ = logits.clone().requires_grad_(True)
    ref = F.cross_entropy(lr_, y)
    ref.backward()
    assert abs(float(loss) - float(ref)) < 1e-3
    assert int(correct) == int((logits.argmax(1) == y).sum())
    assert rel_err(dl, lr_.grad) < 1e-2


def test_sgd_matches_torch(native_ext):
    from ddp_amd.optim import FusedSGD
    torch.manual_seed(0)
    ps = [torch.nn.Parameter(torch.randn(s, device=DEV)) for s in [(17,), (64, 3, 3, 3), (5, 7)]]
    ref = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    opt = FusedSGD(ps, lr=0.1, momentum=0.9, weight_decay=1e-4)
    ropt = torch.optim.SGD(ref, lr=0.1, momentum=0.9, weight_decay=1e-4)
    for it in range(3):
        gs = [torch.randn_like(p) for p in ps]
        opt.zero_grad()
        for p, g in zip(ps, gs):
            p.grad.copy_(g)
        for p, g in zip(ref, gs):
            p.grad = g.clone()
        opt.step()
        ropt.step()
    for p, r in zip(ps, ref):
        assert torch.allclose(p, r, rtol=1e-5, atol=1e-6)


def test_pack_weights(native_ext):
    from ddp_amd.ops.layers import ConvBNActSpec
    conv = torch.nn.Conv2d(3, 64, 3, padding=1).to(DEV)
    spec = ConvBNActSpec(conv, None, cin_pad=8)
    spec.maybe_pack()
    w = conv.weight.detach()
    exp = torch.zeros(64, 3, 3, 8, device=DEV)
    exp[..., :3] = w.permute(0, 2, 3, 1)
    assert torch.equal(spec.wc.float(), exp.to(torch.bfloat16).float())
    conv2 = torch.nn.Conv2d(64, 128, 3, padding=1).to(DEV)
    s2 = ConvBNActSpec(conv2, None)
    s2.maybe_pack()
    assert s2.wt is None  # dgrad reads Wc k-major: no transposed copy
    assert torch.equal(s2.wc.float(), conv2.weight.detach().permute(0, 2, 3, 1).to(torch.bfloat16).float())
    # [K][R][S][C] fp32 master (GPU arena layout)
    conv3 = torch.nn.Conv2d(3, 64, 3, padding=1).to(DEV)
    conv3.weight.data = conv3.weight.data.contiguous(memory_format=torch.channels_last)
    s3 = ConvBNActSpec(conv3, None, cin_pad=8)
    s3.maybe_pack()
    exp = torch.zeros(64, 3, 3, 8, device=DEV)
    exp[..., :3] = conv3.weight.detach().permute(0, 2, 3, 1)
    assert torch.equal(s3.wc.float(), exp.to(torch.bfloat16).float())


def test_synthetic_and_augment_match_cpu(native_ext):
    import numpy as np
    from ddp_amd.data import SyntheticCIFAR10, DeviceLoader, augment_cpu
    ds = SyntheticCIFAR10(True, n=300)
    imgs_c, labels_c = ds.cpu_arrays()
    imgs_g, labels_g = ds.device_arrays(DEV)
    assert np.array_equal(imgs_g.cpu().numpy(), imgs_c)
    assert np.array_equal(labels_g.cpu().numpy(), labels_c)
    loader = DeviceLoader(ds, 50, DEV, num_replicas=2, rank=1, epoch=3)
    x, y = loader.batch(10, 50)
    idx = loader.idx[10:60].cpu().numpy()
    ref = augment_cpu(imgs_c, idx, ds.seed, 3, train=True)
    got = x[..., :3].permute(0, 3, 1, 2).float().cpu()
    # fp32 op order differs from numpy: allow one bf16 ulp on rounding ties
    assert torch.allclose(got, ref.to(torch.bfloat16).float(), rtol=8e-3, atol=1e-2)
    assert torch.all(x[..., 3:] == 0)
    assert torch.equal(y.cpu(), torch.from_numpy(labels_c[idx]))


@pytest.mark.parametrize("shape,cpad", [((64, 3, 3, 3), 8), ((128, 64, 3, 3), None),
                                        ((256, 64, 1, 1), None), ((64, 3, 7, 7), 8),
                                        ((48, 40, 3, 3), None)])
def test_fused_sgd_repacks_conv_weights(native_ext, shape, cpad):
    from ddp_amd.ops.layers import ConvBNActSpec
    from ddp_amd.optim import FusedSGD
    K, Cr, R, S = shape
    conv = torch.nn.Conv2d(Cr, K, R, padding=R // 2).to(DEV)
    bn = torch.nn.BatchNorm2d(K).to(DEV)
    spec = ConvBNActSpec(conv, bn, cin_pad=cpad)
    params = list(conv.parameters()) + list(bn.parameters())
    ref = [torch.nn.Parameter(p.detach().clone()) for p in params]
    opt = FusedSGD(params, lr=0.1, momentum=0.9, weight_decay=1e-4)
    ropt = torch.optim.SGD(ref, lr=0.1, momentum=0.9, weight_decay=1e-4)
    for _ in range(2):
        gs = [torch.randn_like(p) for p in params]
        opt.zero_grad()
        for p, g in zip(params, gs):
            p.grad.copy_(g)
        for p, g in zip(ref, gs):
            p.grad = g.clone()
        opt.step()
        ropt.step()
    torch.cuda.synchronize()
    for p, r in zip(params, ref):
        assert torch.allclose(p, r, rtol=1e-5, atol=1e-6)
    w = conv.weight.detach()
    C = spec.C
    exp_wc = torch.zeros(K, R, S, C, device=DEV)
    exp_wc[..., :Cr] = w.permute(0, 2, 3, 1)
    assert torch.equal(spec.wc.float(), exp_wc.to(torch.bfloat16).float())
    if spec.wt is not None:
        assert torch.equal(spec.wt.float(), w.permute(1, 2, 3, 0).to(torch.bfloat16).float())


def test_maxpool3x3s2_and_avgpool(native_ext):
    from ddp_amd.ops.layers import max_pool, global_avg_pool
    x = bf(torch.randn(4, 64, 15, 15, device=DEV))
    xn = x.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16).requires_grad_(True)
    y = max_pool(xn, 3, 2, 1)
    xr = x.clone().requires_grad_(True)
    yr = F.max_pool2d(xr, 3, 2, 1)
    assert torch.equal(y.permute(0, 3, 1, 2).float(), yr)
    g = bf(torch.randn_like(yr))
    y.backward(g.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16))
    yr.backward(g)
    assert rel_err(xn.grad.permute(0, 3, 1, 2), xr.grad) < 1e-2
    a = global_avg_pool(xn.detach().requires_grad_(True))
    ar = x.mean((2, 3))
    assert rel_err(a, ar) < 1e-2
    # ResNet head shape (7x7, 2048 channels) and an odd one: 4 waves split the pixels
    for (n, c, hw) in ((8, 2048, 7), (3, 24, 5)):
        x2 = bf(torch.randn(n, c, hw, hw, device=DEV))
        a2 = global_avg_pool(x2.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16))
        assert rel_err(a2, x2.mean((2, 3))) < 1e-2


@pytest.mark.parametrize("B,J", [(256, 1000), (37, 10), (64, 17)])
def test_colsum_bias_grad(native_ext, B, J):
    """Bias gradient of the GEMM Linear: db += column sums of bf16 dlogits (pool.hip colsum)."""
    from ddp_amd.ops.common import ptr, stream_handle
    dl = bf(torch.randn(B, J, device=DEV)).to(torch.bfloat16)
    db = torch.full((J,), 0.5, device=DEV)
    native_ext.colsum(ptr(dl), B, J, ptr(db), stream_handle())
    torch.cuda.synchronize()
    assert torch.allclose(db, 0.5 + dl.float().sum(0), rtol=1e-5, atol=1e-4)


def test_fused_sgd_zero_grad_and_counter(native_ext):
    """step(zero_grad=True, counter=...) == step() + zero_grad() + counter += delta."""
    from ddp_amd.optim import FusedSGD
    from ddp_amd.ops.layers import ConvBNActSpec
    torch.manual_seed(0)
    conv = torch.nn.Conv2d(64, 128, 3, padding=1).to(DEV)
    ConvBNActSpec(conv, None)  # packed conv weight: exercises the tile path too
    ps = list(conv.parameters()) + [torch.nn.Parameter(torch.randn(33, device=DEV))]
    ref = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    opt = FusedSGD(ps, lr=0.1, momentum=0.9, weight_decay=1e-4)
    ropt = torch.optim.SGD(ref, lr=0.1, momentum=0.9, weight_decay=1e-4)
    cnt = torch.zeros(1, dtype=torch.int32, device=DEV)
    for _ in range(2):
        gs = [torch.randn_like(p) for p in ps]
        for p, g in zip(ps, gs):
            p.grad.copy_(g)
        for p, g in zip(ref, gs):
            p.grad = g.clone()
        opt.step(zero_grad=True, counter=(cnt.data_ptr(), 3))
        ropt.step()
        torch.cuda.synchronize()
        assert all(float(p.grad.abs().max()) == 0.0 for p in ps)
    assert int(cnt.item()) == 6
    for p, r in zip(ps, ref):
        assert torch.allclose(p, r, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("case", [(8, 512, 2, 2, 512, 3, 1, 1), (4, 64, 16, 16, 128, 3, 1, 1),
                                  (4, 64, 15, 15, 32, 3, 2, 1), (2, 128, 14, 14, 256, 1, 1, 0)])
def test_conv_splitk_forced(native_ext, case):
    """Forced split-K (4 splits: fp32 slabs + finish kernels, bias, bf16 rounding, BN statistics
    in the finish) for FWD / DGRAD / WGRAD against fp32 PyTorch."""
    from ddp_amd.ops.common import ptr, stream_handle, workspace
    N, Cin, H, W, K, R, stride, pad = case
    conv, spec, x, xn = _conv_setup(N, Cin, H, W, K, R, stride, pad)
    ws = workspace(xn.device)
    g = spec.geom(N, H, W)
    P, Q = g[9], g[10]
    z = torch.empty(N, P, Q, K, dtype=torch.bfloat16, device=DEV)
    stats = torch.zeros(16 * 2 * K, device=DEV)
    native_ext.conv_fwd(g, ptr(xn), ptr(spec.wc), ptr(conv.bias), ptr(z), ptr(stats), ptr(ws),
                        ws.numel(), 4, stream_handle())
    dz = bf(torch.randn(N, K, P, Q, device=DEV))
    dzn = dz.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16)
    dx = torch.empty_like(xn)
    native_ext.conv_dgrad(g, ptr(dzn), ptr(spec.wc), ptr(dx), ptr(ws), ws.numel(), 4,
                          stream_handle())
    dw = torch.zeros_like(conv.weight)
    native_ext.conv_wgrad(g, ptr(dzn), ptr(xn), ptr(dw), ptr(ws), ws.numel(), 4, stream_handle())
    torch.cuda.synchronize()
    ref = F.conv2d(x, conv.weight, conv.bias, stride, pad).permute(0, 2, 3, 1)
    assert rel_err(z, ref) < 1e-2
    zf = z.float().reshape(-1, K)
    st = stats.view(16, 2 * K).sum(0)
    assert torch.allclose(st[:K], zf.sum(0), rtol=1e-3, atol=1e-2)
    assert torch.allclose(st[K:], (zf * zf).sum(0), rtol=1e-3, atol=1e-2)
    xr = x.clone().requires_grad_(True)
    wr = conv.weight.detach().clone().requires_grad_(True)
    F.conv2d(xr, wr, None, stride, pad).backward(dz)
    assert rel_err(dx.permute(0, 3, 1, 2), xr.grad) < 1e-2
    assert rel_err(dw, wr.grad) < 1e-2


@pytest.mark.parametrize("N,C,H,K,pool", [(32, 512, 4, 512, True), (32, 512, 2, 512, False),
                                          (8, 256, 8, 512, True), (64, 256, 4, 512, False),
                                          (16, 512, 8, 512, True)])
def test_conv_splitk_finish_bn_fwd(native_ext, N, C, H, K, pool):
    """BatchNorm(+ReLU, +2x2 pool) forward fused into a small conv GEMM's split-K finish
    (conv_igemm.hip splitk_finish_bnfwd_kernel): y, z and the coefficient table against the fp32
    PyTorch reference, and against the separate finish + bn_act_fwd path."""
    from ddp_amd.ops.common import ptr, stream_handle, workspace
    nat = native_ext
    conv, spec, x, xn = _conv_setup(N, C, H, H, K, 3, 1, 1)
    gamma = torch.rand(K, device=DEV) + 0.5
    beta = torch.randn(K, device=DEV) * 0.1
    Ho = H // 2 if pool else H
    g = spec.geom(N, H, H)
    ws = workspace(torch.device(DEV))
    s = stream_handle()
    y = torch.empty(N, Ho, Ho, K, device=DEV, dtype=torch.bfloat16)
    z = torch.empty(N, H, H, K, device=DEV, dtype=torch.bfloat16)
    coef = torch.zeros(6 * K, device=DEV)
    stats = torch.zeros(16 * 2 * K, device=DEV)
    nat.conv_tune_set(0, N * H * H, K, 9 * C, 3, 4, 2)  # force split-K 4 (64x64 tiles)
    nat.conv_bn_fuse_rows(1024)  # every case fused (the shipped limit is 128 rows)
    try:
        fused = nat.conv_fwd_bn(g, ptr(xn), ptr(spec.wc), ptr(conv.bias), ptr(z), ptr(stats),
                                ptr(ws), ws.numel(), s,
                                (ptr(gamma), ptr(beta), 1e-5, 1, int(pool), ptr(coef), ptr(y), H, H))
        # the unfused path on the same operands
        z2 = torch.empty_like(z)
        stats2 = torch.zeros_like(stats)
        nat.conv_fwd(g, ptr(xn), ptr(spec.wc), ptr(conv.bias), ptr(z2), ptr(stats2), ptr(ws),
                     ws.numel(), 0, s)
    finally:
        from ddp_amd.ops.common import load_conv_tuning
        load_conv_tuning(nat)  # back to the shipped table
        nat.conv_bn_fuse_rows(128)
    assert fused, "the split-K GEMM must take the fused BatchNorm finish"
    y2 = torch.empty_like(y)
    coef2 = torch.zeros_like(coef)
    nat.bn_act_fwd(N, H, H, K, int(pool), 1, 1e-5, ptr(z2), 0, ptr(stats2), ptr(gamma),
                   ptr(beta), ptr(y2), s, coef=ptr(coef2))
    torch.cuda.synchronize()
    assert torch.equal(z, z2)  # same slabs, same per-element summation order
    assert torch.allclose(coef[:4 * K], coef2[:4 * K], rtol=1e-4, atol=1e-5)
    assert (y.float() - y2.float()).abs().max() <= 2e-2 * y2.float().abs().max()
    zr = F.conv2d(x, conv.weight, conv.bias, 1, 1)
    ref = _bn_ref(zr, gamma, beta, 1e-5, True, pool, None)
    assert rel_err(y.permute(0, 3, 1, 2), ref) < 1e-2


@pytest.mark.parametrize("tile", [0, 1, 2, 3, 4, 5])
@pytest.mark.parametrize("splits", [1, 3])
@pytest.mark.parametrize("staged", [0, 1])
@pytest.mark.parametrize("case", [(4, 64, 14, 14, 256, 1, 1, 0), (4, 256, 14, 14, 64, 1, 1, 0),
                                  (2, 64, 12, 12, 64, 3, 1, 1)])
def test_conv_dgrad_deferred_branch(native_ext, case, staged, splits, tile):
    """Accumulating dgrad onto a DEFERRED first branch (ResNet identity blocks, GradLink.defer):
    dx = dgrad + (bit ? acc_dy : 0) with the ReLU mask bits of the residual BatchNorm — every
    epilogue (direct fragment stores, LDS-staged rows, split-K finish) must give exactly what
    the classic accumulate gives on the stored masked gradient."""
    from ddp_amd.ops.common import ptr, stream_handle, workspace
    from ddp_amd.ops.layers import _masked
    N, Cin, H, W, K, R, stride, pad = case
    conv, spec, x, xn = _conv_setup(N, Cin, H, W, K, R, stride, pad)
    ws = workspace(xn.device)
    g = spec.geom(N, H, W)
    P, Q = g[9], g[10]
    dzn = bf(torch.randn(N, K, P, Q, device=DEV)).permute(0, 2, 3, 1).contiguous().to(torch.bfloat16)
    acc_dy = bf(torch.randn(N, H, W, Cin, device=DEV)).to(torch.bfloat16)
    mask = torch.randint(0, 256, (N, H, W, Cin // 8), dtype=torch.uint8, device=DEV)
    stored = _masked(acc_dy, mask)
    assert torch.equal(stored.float() != 0, ((mask.unsqueeze(-1).long() >> torch.arange(
        8, device=DEV)) & 1).reshape(acc_dy.shape).bool() & (acc_dy.float() != 0))
    native_ext.conv_force_tile(tile, 0)
    native_ext.conv_epi_stage_set(staged)
    try:
        dxa = stored.clone()
        native_ext.conv_dgrad(g, ptr(dzn), ptr(spec.wc), ptr(dxa), ptr(ws), ws.numel(), splits,
                              stream_handle(), accumulate=1)
        dxd = torch.full_like(xn, float("nan"))  # written, never read
        native_ext.conv_dgrad(g, ptr(dzn), ptr(spec.wc), ptr(dxd), ptr(ws), ws.numel(), splits,
                              stream_handle(), accumulate=1, acc_dy=ptr(acc_dy),
                              acc_mask=ptr(mask))
        torch.cuda.synchronize()
    finally:
        native_ext.conv_force_tile(0, 0)
        native_ext.conv_epi_stage_set(1)
    assert torch.equal(dxd, dxa)
    xr = x.clone().requires_grad_(True)
    F.conv2d(xr, conv.weight.detach(), None, stride, pad).backward(
        dzn.float().permute(0, 3, 1, 2))
    ref = xr.grad.permute(0, 2, 3, 1) + stored.float()
    assert rel_err(dxd, ref) < 1e-2


@pytest.mark.parametrize("tile", [1, 2, 3, 5])  # the tiles the tuned table uses (not 64x64)
@pytest.mark.parametrize("case", [(4, 64, 28, 28, 256, 1, 1, 0), (4, 256, 28, 28, 64, 1, 1, 0),
                                  (3, 64, 21, 21, 128, 1, 2, 0), (2, 64, 14, 14, 128, 3, 1, 1)])
def test_conv_staged_epilogue(native_ext, case, tile):
    """LDS-staged FWD / DGRAD epilogue (conv_igemm.hip epi_stage: bf16 tile through the idle
    operand ring, 16-B row stores, BN statistics per 8-channel chunk) on every big tile, without
    split-K: output bit-identical to the direct fragment stores (same fp32 sums, same rounding),
    statistics and the accumulating second-branch dgrad (dx += ...) against fp32 PyTorch; the
    strided case runs the phase-decomposed dgrad (row -> input pixel remap in the store)."""
    from ddp_amd.ops.common import ptr, stream_handle, workspace
    N, Cin, H, W, K, R, stride, pad = case
    conv, spec, x, xn = _conv_setup(N, Cin, H, W, K, R, stride, pad)
    ws = workspace(xn.device)
    g = spec.geom(N, H, W)
    P, Q = g[9], g[10]
    dz = bf(torch.randn(N, K, P, Q, device=DEV))
    dzn = dz.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16)
    prior = bf(torch.randn(N, H, W, Cin, device=DEV)).to(torch.bfloat16)
    out = {}
    native_ext.conv_force_tile(tile, 0)
    try:
        for staged in (0, 1):
            native_ext.conv_epi_stage_set(staged)
            z = torch.empty(N, P, Q, K, dtype=torch.bfloat16, device=DEV)
            stats = torch.zeros(16 * 2 * K, device=DEV)
            native_ext.conv_fwd(g, ptr(xn), ptr(spec.wc), ptr(conv.bias), ptr(z), ptr(stats),
                                ptr(ws), ws.numel(), 1, stream_handle())
            dx = torch.empty_like(xn)
            native_ext.conv_dgrad(g, ptr(dzn), ptr(spec.wc), ptr(dx), ptr(ws), ws.numel(), 1,
                                  stream_handle())
            dxa = prior.clone()
            native_ext.conv_dgrad(g, ptr(dzn), ptr(spec.wc), ptr(dxa), ptr(ws), ws.numel(), 1,
                                  stream_handle(), accumulate=1)
            torch.cuda.synchronize()
            out[staged] = (z, stats.view(16, 2 * K).sum(0), dx, dxa)
    finally:
        native_ext.conv_force_tile(0, 0)
        native_ext.conv_epi_stage_set(1)
    (z0, s0, dx0, dxa0), (z1, s1, dx1, dxa1) = out[0], out[1]
    assert torch.equal(z0, z1) and torch.equal(dx0, dx1) and torch.equal(dxa0, dxa1)
    ref = F.conv2d(x, conv.weight, conv.bias, stride, pad).permute(0, 2, 3, 1)
    assert rel_err(z1, ref) < 1e-2
    zf = z1.float().reshape(-1, K)
    assert torch.allclose(s1[:K], zf.sum(0), rtol=1e-3, atol=1e-2)
    assert torch.allclose(s1[K:], (zf * zf).sum(0), rtol=1e-3, atol=1e-2)
    assert torch.allclose(s0, s1, rtol=1e-4, atol=1e-3)
    xr = x.clone().requires_grad_(True)
    F.conv2d(xr, conv.weight.detach(), None, stride, pad).backward(dz)
    assert rel_err(dx1.permute(0, 3, 1, 2), xr.grad) < 1e-2
    assert rel_err(dxa1.float(), xr.grad.permute(0, 2, 3, 1) + prior.float()) < 1e-2


@pytest.mark.parametrize("N,C,H,running", [(4, 64, 16, False), (2, 64, 15, True), (3, 32, 9, False)])
def test_bn_relu_maxpool3_fused(native_ext, N, C, H, running):
    """ResNet stem BatchNorm + ReLU + MaxPool2d(3, 2, 1) in one pass each way (bn_act.hip
    bn_pool3_*): pooled output, running statistics, dz (pooled gradient gathered through the
    window argmax bytes and the recomputed ReLU mask), dgamma / dbeta against fp32 PyTorch."""
    from ddp_amd.ops.common import ptr, stream_handle
    nat = native_ext
    z = bf(torch.randn(N, C, H, H, device=DEV) * 2 + 0.3)
    gamma = torch.rand(C, device=DEV) + 0.5
    beta = torch.randn(C, device=DEV) * 0.1
    zn = z.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16)
    zf = zn.float().reshape(-1, C)
    stats = torch.zeros(16, 2 * C, device=DEV)
    stats[5] = torch.cat([zf.sum(0), (zf * zf).sum(0)])
    Ho = (H - 1) // 2 + 1
    out = torch.empty(N, Ho, Ho, C, device=DEV, dtype=torch.bfloat16)
    idx = torch.empty(N, Ho, Ho, C, device=DEV, dtype=torch.uint8)
    rm = torch.zeros(C, device=DEV) if running else None
    rv = torch.ones(C, device=DEV) if running else None
    coef = torch.empty(6 * C, device=DEV)
    s = stream_handle()
    nat.bn_pool3_fwd(N, H, H, C, 1, 1e-5, ptr(zn), ptr(stats), ptr(gamma), ptr(beta), ptr(out),
                     ptr(idx), s, ptr(rm), ptr(rv), 0.1, 0, ptr(coef))
    zr = z.clone().requires_grad_(True)
    gr = gamma.clone().requires_grad_(True)
    br = beta.clone().requires_grad_(True)
    rm_ref = torch.zeros(C, device=DEV)
    rv_ref = torch.ones(C, device=DEV)
    ref = F.max_pool2d(F.relu(F.batch_norm(zr, rm_ref, rv_ref, gr, br, True, 0.1, 1e-5)), 3, 2, 1)
    assert rel_err(out.permute(0, 3, 1, 2), ref) < 1e-2
    if running:
        assert torch.allclose(rm, rm_ref, rtol=1e-4, atol=1e-5)
        assert torch.allclose(rv, rv_ref, rtol=1e-3, atol=1e-4)
    dout = bf(torch.randn_like(ref))
    ref.backward(dout)
    doutn = dout.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16)
    sums = torch.zeros(16 * 2 * C, device=DEV)
    dz = torch.empty_like(zn)
    dg = torch.zeros(C, device=DEV)
    db = torch.zeros(C, device=DEV)
    nat.bn_pool3_bwd(N, H, H, C, 1, 1e-5, ptr(zn), ptr(doutn), ptr(idx), ptr(sums), ptr(dz),
                     ptr(dg), ptr(db), s, ptr(coef))
    torch.cuda.synchronize()
    assert rel_err(dz.permute(0, 3, 1, 2), zr.grad) < 2e-2
    assert rel_err(dg, gr.grad) < 1e-2
    assert rel_err(db, br.grad) < 1e-2


TILE_NAMES = ["128x128", "128x64", "64x128", "64x64", "256x64", "64x256", "256x128", "128x256"]


@pytest.mark.parametrize("tile", range(8))
@pytest.mark.parametrize("case", [(2, 128, 14, 14, 256, 1, 1, 0), (4, 64, 16, 16, 128, 3, 1, 1),
                                  (2, 256, 8, 8, 512, 3, 1, 1), (2, 64, 15, 15, 64, 3, 2, 1)])
def test_conv_every_tile(native_ext, case, tile):
    """Every implicit-GEMM tile the launcher can select (measured table or conv_force_tile) for
    FWD, DGRAD and WGRAD against fp32 PyTorch — including the 256-wide k-major operand tiles whose
    per-chunk swizzle was wrong before round 4 (conv_igemm.hip swz_row_step). WGRAD never runs
    BN = 256 tiles (tile_ok): forcing them must fall back to a correct tile."""
    from ddp_amd.ops.layers import conv_forward, conv_backward
    N, Cin, H, W, K, R, stride, pad = case
    conv, spec, x, xn = _conv_setup(N, Cin, H, W, K, R, stride, pad)
    P = (H + 2 * pad - R) // stride + 1
    dz = bf(torch.randn(N, K, P, P, device=DEV))
    dzn = dz.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16)
    dw = torch.zeros_like(conv.weight, memory_format=torch.channels_last)
    native_ext.conv_force_tile(tile + 1, 0)
    native_ext.conv_pair_mode(0)  # separate DGRAD / WGRAD launches, each on the forced tile
    import ddp_amd.ops.layers as L
    ctr = L.CONV_TR
    L.CONV_TR = False  # the implicit-GEMM forward, not the tap-reuse kernel
    try:
        z = conv_forward(spec, xn, conv.bias, None)
        dx = conv_backward(spec, xn, dzn, dw, True)
        torch.cuda.synchronize()
    finally:
        L.CONV_TR = ctr
        native_ext.conv_pair_mode(3)
        native_ext.conv_force_tile(0, 0)
    ref = F.conv2d(x, conv.weight, conv.bias, stride, pad).permute(0, 2, 3, 1)
    xr = x.clone().requires_grad_(True)
    wr = conv.weight.detach().clone().requires_grad_(True)
    F.conv2d(xr, wr, None, stride, pad).backward(dz)
    errs = {"fwd": rel_err(z, ref), "dgrad": rel_err(dx.permute(0, 3, 1, 2), xr.grad),
            "wgrad": rel_err(dw, wr.grad)}
    bad = {k: v for k, v in errs.items() if not v < 1e-2}
    assert not bad, f"tile {TILE_NAMES[tile]}: {bad}"


@pytest.mark.parametrize("pair_mode", [0, 3])
@pytest.mark.parametrize("N,C,K", [(32, 512, 512), (256, 512, 512), (64, 128, 256)])
def test_conv_dense2x2(native_ext, N, C, K, pair_mode):
    """3x3 / s1 / p1 convs over 2x2 images as ONE dense GEMM per direction (conv_igemm.hip
    ConvArgs::d2x2: the tap of each (output pixel, input pixel) block read straight from Wc, the
    split-K finish on the 3x3 view): z, the BatchNorm statistics of the rounded z, dx and dW
    against fp32 PyTorch, and against the implicit-GEMM path (dense switched off), separately
    launched (pair mode 0) and as the grouped backward pair (3). VGG-11 layers 6-7
    (/root/reference/part1/model.py:18-23 at 2x2)."""
    from ddp_amd.ops.layers import conv_forward, conv_backward
    nat = native_ext
    conv, spec, x, xn = _conv_setup(N, C, 2, 2, K, 3, 1, 1)
    assert nat.conv_dense2x2_ok(spec.geom(N, 2, 2))
    dz = bf(torch.randn(N, K, 2, 2, device=DEV))
    dzn = dz.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16)
    out = {}
    nat.conv_pair_mode(pair_mode)
    try:
        for dense in (1, 0):
            nat.conv_dense2x2_set(dense)
            stats = torch.zeros(16 * 2 * K, device=DEV)
            dw = torch.zeros_like(conv.weight, memory_format=torch.channels_last)
            z = conv_forward(spec, xn, conv.bias, stats)
            dx = conv_backward(spec, xn, dzn, dw, True)
            torch.cuda.synchronize()
            out[dense] = (z.clone(), stats.view(16, 2 * K).sum(0), dx.clone(), dw.clone())
    finally:
        nat.conv_dense2x2_set(1)
        nat.conv_pair_mode(3)
    ref = F.conv2d(x, conv.weight, conv.bias, 1, 1).permute(0, 2, 3, 1)
    xr = x.clone().requires_grad_(True)
    wr = conv.weight.detach().clone().requires_grad_(True)
    F.conv2d(xr, wr, None, 1, 1).backward(dz)
    for dense in (1, 0):
        z, st, dx, dw = out[dense]
        assert rel_err(z, ref) < 1e-2, (dense, rel_err(z, ref))
        zf = z.float().reshape(-1, K)
        assert torch.allclose(st[:K], zf.sum(0), rtol=1e-3, atol=1e-2), dense
        assert torch.allclose(st[K:], (zf * zf).sum(0), rtol=1e-3, atol=1e-2), dense
        assert rel_err(dx.permute(0, 3, 1, 2), xr.grad) < 1e-2, dense
        assert rel_err(dw, wr.grad) < 1e-2, dense
    assert rel_err(out[1][0], out[0][0]) < 1e-2
    assert rel_err(out[1][2], out[0][2]) < 1e-2


@pytest.mark.parametrize("pair_mode", [0, 3])
@pytest.mark.parametrize("case", [(32, 64, 16, 128, True, False), (8, 128, 8, 256, False, False),
                                  (32, 256, 4, 512, True, False), (4, 64, 32, 64, True, False),
                                  (8, 8, 32, 64, True, True), (4, 64, 14, 128, False, False)])
def test_conv_bwd_after_bn(native_ext, case, pair_mode):
    """The conv backward GEMMs on the dz of a training-mode BatchNorm backward (reduce ->
    finalize -> apply): dx and dW must match fp32 PyTorch through conv -> BN -> ReLU (-> 2x2
    pool), separately launched (pair mode 0) and as the grouped backward pair (3). Covers pooled
    / unpooled BN, the padded input layer (C = 8: wgrad only) and a 14x14 image (partial
    tiles). Reference hot path: /root/reference/part1/model.py:18-27."""
    from ddp_amd.ops.common import ptr, stream_handle
    from ddp_amd.ops.layers import conv_backward
    nat = native_ext
    N, Cin, H, K, pool, first = case
    Creal = 3 if first else Cin
    conv, spec, x, xn = _conv_setup(N, Cin, H, H, K, 3, 1, 1, Creal)
    need_dx = not first
    s = stream_handle()
    with torch.no_grad():  # bf16-valued conv output, NCHW (a leaf for the BN reference below)
        zt = bf(F.conv2d(x, conv.weight, conv.bias, 1, 1))
    zn = zt.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16)
    gamma = torch.rand(K, device=DEV) + 0.5
    beta = torch.randn(K, device=DEV) * 0.1
    zf = zn.float().reshape(-1, K)
    stats = torch.zeros(16, 2 * K, device=DEV)
    stats[0] = torch.cat([zf.sum(0), (zf * zf).sum(0)])
    coef = torch.empty(6 * K, device=DEV)
    Ho = H // 2 if pool else H
    out = torch.empty(N, Ho, Ho, K, device=DEV, dtype=torch.bfloat16)
    nat.bn_act_fwd(N, H, H, K, int(pool), 1, 1e-5, ptr(zn), 0, ptr(stats), ptr(gamma), ptr(beta),
                   ptr(out), s, coef=ptr(coef))
    dout = bf(torch.randn(N, K, Ho, Ho, device=DEV))
    doutn = dout.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16)
    # fp32 reference: BN backward on the same z, then the conv backward on that dz
    zr = zt.clone().requires_grad_(True)
    _bn_ref(zr, gamma, beta, 1e-5, True, pool).backward(dout)
    xr = x.clone().requires_grad_(True)
    wr = conv.weight.detach().clone().requires_grad_(True)
    F.conv2d(xr, wr, None, 1, 1).backward(zr.grad)
    nat.bn_bwd_local_set(0)
    nat.conv_pair_mode(pair_mode)
    try:
        sums = torch.zeros(16 * 2 * K, device=DEV)
        dg = torch.zeros(K, device=DEV)
        db = torch.zeros(K, device=DEV)
        dw = torch.zeros_like(conv.weight, memory_format=torch.channels_last)
        dz = torch.empty_like(zn)
        nat.bn_act_bwd(N, H, H, K, int(pool), 1, 1e-5, ptr(zn), 0, ptr(stats), ptr(gamma),
                       ptr(beta), ptr(doutn), ptr(sums), ptr(dz), 0, ptr(dg), ptr(db), 0,
                       s, ptr(coef))
        dx = conv_backward(spec, xn, dz, dw, need_dx)
        torch.cuda.synchronize()
    finally:
        nat.bn_bwd_local_set(8)
        nat.conv_pair_mode(3)
    assert rel_err(dw, wr.grad) < 2e-2, rel_err(dw, wr.grad)
    if need_dx:
        assert rel_err(dx.permute(0, 3, 1, 2), xr.grad) < 2e-2


@pytest.mark.parametrize("path", ["pair", "separate", "layer0"])
def test_sgd_in_backward_finish(native_ext, path):
    """SGD in the backward (conv_igemm.hip SgdFuse): a registered weight's WGRAD split-K finish
    applies torch.optim.SGD's update (momentum 0.9, wd 1e-4) to the fp32 master and its momentum
    buffer and rewrites the bf16 forward copy, instead of storing the gradient. Checked against
    the unfused backward's gradient + the SGD formula in fp32 PyTorch; dx must be unchanged
    (the DGRAD reads the weights before the update: grouped pair, or DGRAD issued first)."""
    from ddp_amd.ops.layers import conv_backward
    nat = native_ext
    if path == "layer0":
        N, Cin, H, K, Creal, need_dx = 8, 8, 32, 64, 3, False
    else:
        N, Cin, H, K, Creal, need_dx = 8, 64, 16, 128, 64, True
    conv, spec, x, xn = _conv_setup(N, Cin, H, H, K, 3, 1, 1, Creal=Creal)
    dz = bf(torch.randn(N, K, H, H, device=DEV))
    dzn = dz.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16)
    lr, mom, wd = 0.1, 0.9, 1e-4
    mode = {"pair": 2, "separate": 0, "layer0": 3}[path]
    nat.conv_pair_mode(mode)
    if path == "pair":
        nat.conv_pair_force(1, 4)  # WGRAD split 4 ways: a single-group finish
    try:
        dw_ref = torch.zeros_like(conv.weight, memory_format=torch.channels_last)
        dx_ref = conv_backward(spec, xn, dzn, dw_ref, need_dx)
        torch.cuda.synchronize()
        p = conv.weight.detach().clone().contiguous(memory_format=torch.channels_last)
        buf = (torch.randn_like(p) * 1e-3).contiguous(memory_format=torch.channels_last)
        p0, buf0 = p.clone(), buf.clone()
        dw = torch.zeros_like(p)
        nat.sgd_fuse_register(dw.data_ptr(), p.data_ptr(), buf.data_ptr(), spec.wc.data_ptr(),
                              lr, mom, wd, 1.0, 0, clear=1)
        nat.sgd_fuse_begin()
        try:
            dx = conv_backward(spec, xn, dzn, dw, need_dx)
            torch.cuda.synchronize()
            taken = nat.sgd_fuse_taken()
        finally:
            nat.sgd_fuse_register(0, clear=1)
    finally:
        nat.conv_pair_mode(3)
        nat.conv_pair_force(0, 0)
    if need_dx:
        assert torch.equal(dx, dx_ref)
    if path == "pair":  # forced 4-way WGRAD split: one finish group, the update must be taken
        assert taken == [dw.data_ptr()]
    assert taken in ([], [dw.data_ptr()])
    if not taken:  # the finish did not qualify (multi-group / no split): gradient stored
        assert torch.equal(p, p0) and rel_err(dw, dw_ref) < 1e-6
        return
    assert float(dw.abs().max()) == 0.0  # the gradient never reached memory
    d = dw_ref + wd * p0
    b_ref = mom * buf0 + d
    p_ref = p0 - lr * b_ref
    assert torch.allclose(buf, b_ref, rtol=1e-5, atol=1e-7)
    assert torch.allclose(p, p_ref, rtol=1e-6, atol=1e-7)
    # the bf16 forward operand [K][R][S][C] (pad channels untouched = 0)
    wc = spec.wc.view(K, 3, 3, Cin).float()[..., :Creal]
    assert torch.equal(wc, p.permute(0, 2, 3, 1).to(torch.bfloat16).float())


@pytest.mark.parametrize("N", [4, 32])
def test_l0_fused_input_block(native_ext, N):
    """VGG input block with z recomputed (conv_l0.hip): forward y = maxpool(relu(BN(conv(x)))) and
    backward dz = d loss / d z, dgamma, dbeta against fp32 PyTorch autograd of the same block on
    the same bf16-valued operands (z rounded to bf16 as the kernels store/recompute it)."""
    from ddp_amd.ops.common import ptr, stream_handle
    nat = native_ext
    K, H = 64, 32
    conv, spec, x, xn = _conv_setup(N, 8, H, H, K, 3, 1, 1, Creal=3)
    g = spec.geom(N, H, H)
    assert nat.l0_ok(g)
    gamma = torch.rand(K, device=DEV) + 0.5
    beta = torch.randn(K, device=DEV) * 0.1
    eps = 1e-5
    s = stream_handle()
    stats = torch.zeros(16 * 2 * K, device=DEV)
    coef = torch.full((6 * K,), float("nan"), device=DEV)
    y = torch.full((N, H // 2, H // 2, K), float("nan"), device=DEV, dtype=torch.bfloat16)
    code = torch.full((N, H // 2, H // 2, K), 0xEE, device=DEV, dtype=torch.uint8)
    zw = torch.full((N, H // 2, H // 2, K), float("nan"), device=DEV, dtype=torch.bfloat16)
    nat.l0_fwd(g, ptr(xn), ptr(spec.wc), ptr(conv.bias), eps, 1, ptr(stats), ptr(gamma),
               ptr(beta), ptr(coef), ptr(y), ptr(code), ptr(zw), s)
    dy = bf(torch.randn(N, K, H // 2, H // 2, device=DEV))
    dyn = dy.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16)
    sums = torch.zeros(16 * 2 * K, device=DEV)
    dz = torch.full((N, H, H, K), float("nan"), device=DEV, dtype=torch.bfloat16)
    dg = torch.zeros(K, device=DEV)
    db = torch.zeros(K, device=DEV)
    nat.l0_bwd(g, ptr(xn), ptr(spec.wc), ptr(conv.bias), eps, 1, ptr(coef), ptr(dyn), ptr(sums),
               ptr(dz), ptr(dg), ptr(db), ptr(code), ptr(zw), s)
    torch.cuda.synchronize()
    # every pooled value got a verdict: a window position, or 4 = ReLU zeroed the window; the
    # bytes are lane-major ([g][j][v] for channel j*16 + 4g + v), 4 exactly where y is 0
    assert int(code.max()) <= 4
    code_c = code.view(N, H // 2, H // 2, 4, 4, 4).permute(0, 1, 2, 4, 3, 5).reshape(y.shape)
    assert torch.equal(code_c == 4, y == 0)
    # zw: the z of the pixel the code names (any window position where code is 4: all ReLU-cut)
    zp = bf(F.conv2d(x, conv.weight, conv.bias, 1, 1)).permute(0, 2, 3, 1)  # [N][H][W][K]
    win = zp.reshape(N, H // 2, 2, H // 2, 2, K).permute(0, 1, 3, 2, 4, 5).reshape(N, H // 2, H // 2, 4, K)
    sel = code_c.long().clamp(max=3).unsqueeze(3)
    zsel = torch.gather(win, 3, sel).squeeze(3)
    ok = code_c < 4
    # (the kernel's bf16 z may differ from the reference conv's rounding by one bf16 step)
    assert torch.allclose(zw.float()[ok], zsel[ok], rtol=8e-3, atol=1e-2)
    with torch.no_grad():
        z = bf(F.conv2d(x, conv.weight, conv.bias, 1, 1))
    zr = z.clone().requires_grad_(True)
    gr = gamma.clone().requires_grad_(True)
    br = beta.clone().requires_grad_(True)
    ref = F.max_pool2d(F.relu(F.batch_norm(zr, None, None, gr, br, training=True, eps=eps)), 2, 2)
    ref.backward(dy)
    assert not torch.isnan(y.float()).any() and not torch.isnan(dz.float()).any()
    assert rel_err(y.permute(0, 3, 1, 2), ref) < 1e-2
    assert rel_err(dz.permute(0, 3, 1, 2), zr.grad) < 2e-2
    assert rel_err(dg, gr.grad) < 1e-2
    assert rel_err(db, br.grad) < 1e-2
    # the forward statistics are those of the bf16-rounded z
    st = stats.view(16, 2 * K).sum(0)
    zf = z.permute(0, 2, 3, 1).reshape(-1, K)
    assert torch.allclose(st[:K], zf.sum(0), rtol=1e-3, atol=1e-2)
    assert torch.allclose(st[K:], (zf * zf).sum(0), rtol=1e-3, atol=1e-2)
