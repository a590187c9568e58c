"""Fused layer runtimes and autograd Functions over the gfx950 kernels.

``ConvBNAct`` is the VGG/ResNet building block
    Conv2d(+bias) -> BatchNorm2d (batch statistics) -> [+ residual] -> ReLU -> [MaxPool 2x2]
executed as two kernels forward (implicit-GEMM conv with the BN statistics fused into its
epilogue, then one streaming BN/ReLU/pool pass) and four backward (BN reduce, BN apply,
conv wgrad, conv dgrad). Parameter gradients are accumulated straight into ``param.grad``
(views into the flat gradient arena) and announced through ``common.grad_ready`` so the DDP
reducer can launch bucket all-reduces while the rest of the backward is still running.

Reference parity: part1/model.py:11-27 (the Sequential it fuses) and SURVEY.md §2.D kernel list.
Activations between blocks are NHWC bf16; the first conv's input is zero-padded 3 -> 8 channels.
"""
import torch

from .common import native, ptr, stream_handle, check, grad_ready, ensure_grad

BF16 = torch.bfloat16
F32 = torch.float32


def _pad8(c):
    return (c + 7) // 8 * 8


class ConvBNActSpec:
    """Static per-layer runtime state: geometry, packed bf16 weight copies, flags."""

    def __init__(self, conv, bn, relu=True, pool=False, cin_pad=None, residual=False):
        K, Cr, R, S = conv.weight.shape
        if conv.groups != 1 or conv.dilation != (1, 1):
            raise ValueError("grouped/dilated conv not supported")
        if conv.stride[0] != conv.stride[1] or conv.padding[0] != conv.padding[1]:
            raise ValueError("only square stride/padding supported")
        if K % 8:
            raise ValueError("output channels must be a multiple of 8")
        self.conv, self.bn = conv, bn
        self.K, self.Cr, self.R, self.S = K, Cr, R, S
        self.C = cin_pad if cin_pad is not None else _pad8(Cr)
        self.stride, self.pad = conv.stride[0], conv.padding[0]
        self.relu, self.pool, self.residual = relu, pool, residual
        self.eps = float(bn.eps) if bn is not None else 1e-5
        dev = conv.weight.device
        self.wc = torch.empty(K, R, S, self.C, dtype=BF16, device=dev)
        self.wt = torch.empty(self.C, R, S, K, dtype=BF16, device=dev) if self.C == Cr else None
        self._packed_version = None
        conv.weight._ddp_amd_pack = self.pack_desc  # the fused optimizer repacks after its step

    def pack_desc(self):
        return (ptr(self.conv.weight), ptr(self.wc), ptr(self.wt), self.K, self.Cr, self.C,
                self.R, self.S)

    def maybe_pack(self):
        w = self.conv.weight
        key = (w.data_ptr(), w._version)
        if key != self._packed_version:
            native().pack_conv_weights([self.pack_desc()], stream_handle())
            self._packed_version = key

    def out_hw(self, H, W):
        P = (H + 2 * self.pad - self.R) // self.stride + 1
        Q = (W + 2 * self.pad - self.S) // self.stride + 1
        return P, Q

    def geom(self, N, H, W):
        P, Q = self.out_hw(H, W)
        return (N, H, W, self.C, self.K, self.R, self.S, self.stride, self.pad, P, Q, self.Cr)


# split-K workspaces are only needed when the GEMM output is small (few tiles)
_WS_LIMIT = 8 << 20


def _ws_for(elems, device):
    if elems * 4 > _WS_LIMIT:
        return None
    return torch.empty(elems, dtype=F32, device=device)


def conv_forward(spec, x, bias=None, stats=None):
    """z = conv(x) + bias (bf16 NHWC); stats[2K] += per-channel sum / sumsq of z."""
    N, H, W, C = x.shape
    check(x, BF16, name="conv input")
    if C != spec.C:
        raise ValueError(f"conv input has {C} channels, layer expects {spec.C}")
    g = spec.geom(N, H, W)
    P, Q = g[9], g[10]
    z = torch.empty(N, P, Q, spec.K, dtype=BF16, device=x.device)
    ws = _ws_for(N * P * Q * spec.K, x.device)
    native().conv_fwd(g, ptr(x), ptr(spec.wc), ptr(bias), ptr(z), ptr(stats), ptr(ws), 0,
                      stream_handle())
    return z


def conv_backward(spec, x, dz, dweight, need_dx):
    N, H, W, C = x.shape
    g = spec.geom(N, H, W)
    s = stream_handle()
    native().conv_wgrad(g, ptr(dz), ptr(x), ptr(dweight), 0, s)
    if not need_dx:
        return None
    if spec.wt is None:
        raise RuntimeError("dgrad requested for a channel-padded input layer")
    dx = torch.empty_like(x)
    ws = _ws_for(N * H * W * spec.C, x.device)
    native().conv_dgrad(g, ptr(dz), ptr(spec.wt), ptr(dx), ptr(ws), 0, s)
    return dx


class _ConvBNActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, gamma, beta, residual, spec):
        spec.maybe_pack()
        N, H, W, _ = x.shape
        stats = torch.zeros(2 * spec.K, dtype=F32, device=x.device)
        z = conv_forward(spec, x, bias, stats)
        P, Q = z.shape[1], z.shape[2]
        Ho, Wo = (P // 2, Q // 2) if spec.pool else (P, Q)
        y = torch.empty(N, Ho, Wo, spec.K, dtype=BF16, device=x.device)
        if residual is not None:
            check(residual, BF16, (N, P, Q, spec.K), "residual")
        native().bn_act_fwd(N, P, Q, spec.K, int(spec.pool), int(spec.relu), spec.eps, ptr(z),
                            ptr(residual), ptr(stats), ptr(gamma), ptr(beta), ptr(y),
                            stream_handle())
        ctx.spec = spec
        ctx.has_res = residual is not None
        ctx.save_for_backward(x, z, stats, weight, bias, gamma, beta, residual)
        return y

    @staticmethod
    def backward(ctx, dy):
        spec = ctx.spec
        x, z, stats, weight, bias, gamma, beta, residual = ctx.saved_tensors
        dy = dy.contiguous()
        N, P, Q, K = z.shape
        dz = torch.empty_like(z)
        sums = torch.empty(2 * K, dtype=F32, device=z.device)
        dres = torch.empty_like(z) if (ctx.has_res and ctx.needs_input_grad[5]) else None
        gw = ensure_grad(weight)
        gb = ensure_grad(bias) if bias is not None else None
        gg = ensure_grad(gamma)
        gbt = ensure_grad(beta)
        native().bn_act_bwd(N, P, Q, K, int(spec.pool), int(spec.relu), spec.eps, ptr(z),
                            ptr(residual), ptr(stats), ptr(gamma), ptr(beta), ptr(dy), ptr(sums),
                            ptr(dz), ptr(dres), ptr(gg), ptr(gbt), ptr(gb), stream_handle())
        grad_ready([gamma, beta, bias])
        dx = conv_backward(spec, x, dz, gw, ctx.needs_input_grad[0])
        grad_ready([weight])
        return dx, None, None, None, None, dres, None


def conv_bn_act(x, spec, residual=None):
    conv, bn = spec.conv, spec.bn
    return _ConvBNActFn.apply(x, conv.weight, conv.bias, bn.weight, bn.bias, residual, spec)


# ------------------------------------------------------------------ classifier head
class _LinearSmallFn(torch.autograd.Function):
    """Linear with few outputs (J <= 16): bf16 [B, F] -> fp32 logits [B, J]."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        B, F = x.shape
        J = weight.shape[0]
        check(x, BF16, name="linear input")
        logits = torch.empty(B, J, dtype=F32, device=x.device)
        native().linear_ce_fwd(ptr(x), ptr(weight), ptr(bias), 0, B, F, J, ptr(logits), 0, 0, 0,
                               stream_handle())
        ctx.save_for_backward(x, weight, bias)
        return logits

    @staticmethod
    def backward(ctx, dlogits):
        x, weight, bias = ctx.saved_tensors
        B, F = x.shape
        J = weight.shape[0]
        dlogits = dlogits.contiguous().float()
        gw = ensure_grad(weight)
        gb = ensure_grad(bias) if bias is not None else None
        dx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        native().linear_bwd(ptr(dlogits), ptr(x), ptr(weight), B, F, J, 0, ptr(dx), ptr(gw),
                            ptr(gb), stream_handle())
        grad_ready([weight, bias])
        return dx, None, None


def linear_small(x, linear):
    if linear.weight.shape[0] > 16:
        raise ValueError("linear_small supports at most 16 outputs")
    return _LinearSmallFn.apply(x, linear.weight, linear.bias)


class _CrossEntropyFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels):
        B, J = logits.shape
        logits = logits.contiguous()
        check(logits, F32, name="logits")
        labels = labels.to(torch.int64).contiguous()
        loss = torch.zeros((), dtype=F32, device=logits.device)
        dl = torch.empty(B, J, dtype=F32, device=logits.device)
        native().softmax_ce(ptr(logits), 0, ptr(labels), B, J, ptr(loss), 0, ptr(dl), 0,
                            stream_handle())
        ctx.save_for_backward(dl)
        return loss

    @staticmethod
    def backward(ctx, g):
        (dl,) = ctx.saved_tensors
        return dl * g, None


def cross_entropy(logits, labels):
    """Mean softmax cross-entropy (reference: nn.CrossEntropyLoss(), part1/main.py:119)."""
    return _CrossEntropyFn.apply(logits, labels)


def to_nhwc_input(x, cpad=8):
    """NCHW fp32 image batch -> NHWC bf16 with channels zero-padded to ``cpad``."""
    if x.dtype == BF16 and x.dim() == 4 and x.shape[-1] == cpad:
        return x.contiguous()
    x = x.contiguous().float()
    N, C, H, W = x.shape
    out = torch.empty(N, H, W, cpad, dtype=BF16, device=x.device)
    native().nchw_to_nhwc(ptr(x), N, C, H, W, cpad, ptr(out), stream_handle())
    return out
