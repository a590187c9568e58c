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

from .common import (native, ptr, stream_handle, check, grad_ready, ensure_grad, workspace,
                     step_scratch, weight_krsc, stat_replicas)
from . import common as _common

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
        # ResNet stem: BatchNorm + ReLU + MaxPool2d(3, 2, 1) fused (bn_act.hip bn_pool3_*; the
        # pre-pool activation and its gradient are never materialised). Set by models/resnet.py
        self.maxpool3 = False
        self.eps = float(bn.eps) if bn is not None else 1e-5
        dev = conv.weight.device
        self.wc = torch.empty(K, R, S, self.C, dtype=BF16, device=dev)
        # transposed copy [C][R][S][K]: none. The backward-data GEMM reads Wc k-major through
        # transposing LDS reads (ds_read_b64_tr_b16); the optimizer's repack keeps the slot
        self.wt = None
        self._packed_version = None
        conv.weight._ddp_amd_pack = self.pack_desc  # the fused optimizer repacks after its step
        # per-step zeroed accumulators (StepScratch): BN statistics replicas + BN-backward sums
        sc = step_scratch(dev)
        self.scratch = sc
        nrep = stat_replicas()
        self.stats = sc.take(nrep * 2 * K)[:nrep * 2 * K]
        sums = sc.take(nrep * 2 * K + 64)
        self.sums = sums[:nrep * 2 * K]
        # per-layer BN coefficient table [6][K] (scale, shift, mean, invstd | k1, k2): written
        # by the forward's finalize kernel, read by the backward (one use per step per layer)
        self.coef = torch.empty(6 * K, dtype=F32, device=dev)
        # BnBwdFuse chaining (VGG): ``prev`` is the Conv->BN->ReLU(->pool) block that produces
        # this block's input; this block's dgrad accumulates prev's BatchNorm-backward sums in
        # its epilogue and sets ``prev.sums_ready`` so prev's backward skips its reduce pass
        self.prev = None
        self.next = None  # the block consuming this block's output (VGG chain)
        # this forward's output y when its BN + ReLU (+ pool) is deferred into the next block's
        # conv (conv_tr.hip fused input): (y, pool) — the next block's forward computes y while
        # loading its input patch, or materialises it with bn_act_fwd if it cannot
        self.deferred = None
        self.fwd_z = None
        self.sums_ready = False
        # set by the next block's backward when its dgrad finish completed this block's BN
        # backward (BN_BWD_APPLY_FUSE): (gradient at this block's conv output, the conv output
        # z of the forward it belongs to). The gradient the next block then hands autograd for
        # this block's output is NOT materialised (uninitialised memory, also as a pipelined
        # step's leaf.grad): this block's backward must take dz_fused instead, and checks that
        # it belongs to the same forward; every forward clears it.
        self.dz_fused = None

    def pack_desc(self):
        w = self.conv.weight
        return (ptr(w), ptr(self.wc), ptr(self.wt), self.K, self.Cr, self.C,
                self.R, self.S, weight_krsc(w))

    def rebind_wc(self, flat):
        """Make the bf16 operand copy a view of ``flat`` (same element order as Wc; the sharded
        update's shadow arena, parallel/zero.py ShardedBf16Update). The next maybe_pack()
        rebuilds it from the fp32 master."""
        if flat.dtype != BF16 or flat.numel() != self.wc.numel():
            raise ValueError("operand view must be bf16 with the operand copy's element count")
        self.wc = flat.view(self.wc.shape)
        self._packed_version = None

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

    def geom(self, N, H, W, wkrsc=0):
        P, Q = self.out_hw(H, W)
        return (N, H, W, self.C, self.K, self.R, self.S, self.stride, self.pad, P, Q, self.Cr,
                wkrsc)


def _fin_args(prev, y):
    """Fused-input tuple of conv_fwd_tr for the preceding block ``prev`` whose output is y."""
    bn = prev.bn
    return (ptr(prev.fwd_z), ptr(prev.stats), ptr(bn.weight), ptr(bn.bias), prev.eps,
            int(prev.relu), int(prev.pool), ptr(prev.coef), ptr(y))


def _bn_act_fwd_now(spec, z, y):
    """The (deferred) BatchNorm + ReLU (+ pool) forward of ``spec`` as its own launch."""
    N, P, Q, K = z.shape
    bn = spec.bn
    native().bn_act_fwd(N, P, Q, K, int(spec.pool), int(spec.relu), spec.eps, ptr(z), 0,
                        ptr(spec.stats), ptr(bn.weight), ptr(bn.bias), ptr(y), stream_handle(),
                        0, 0, float(bn.momentum if bn.momentum is not None else 0.1), 0,
                        ptr(spec.coef))


def conv_forward(spec, x, bias=None, stats=None, bn_fuse=None, fin=None):
    """z = conv(x) + bias (bf16 NHWC); stats[16][2][K] += per-channel sum / sumsq of z
    (accumulated into stat_replicas() replicas; the consumer sums them).

    ``bn_fuse`` = (gamma, beta, eps, relu, pool, coef, y, P, Q) pointers/values: when the GEMM
    runs split-K and is small (the strong-scaling batches' deep layers), its finish kernel also
    computes the BatchNorm forward into y and the coefficient table (conv_igemm.hip
    splitk_finish_bnfwd_kernel). Returns (z, fused) then; plain z otherwise.

    ``fin`` = the preceding block whose BatchNorm + ReLU (+ pool) was deferred (x is its
    unwritten output): the tap-reuse kernel computes x while loading its patch (and writes it);
    when that kernel does not serve the shape, x is materialised first by bn_act_fwd."""
    N, H, W, C = x.shape
    check(x, BF16, name="conv input")
    if C != spec.C:
        raise ValueError(f"conv input has {C} channels, layer expects {spec.C}")
    g = spec.geom(N, H, W)
    P, Q = g[9], g[10]
    z = torch.empty(N, P, Q, spec.K, dtype=BF16, device=x.device)
    if spec.C == 8 and native().conv_fwd_smallk(g, ptr(x), ptr(spec.wc), ptr(bias), ptr(z),
                                                ptr(stats), stream_handle()):
        # input layer (3 channels padded to 8): direct MFMA kernel, conv_smallk.hip
        return (z, False) if bn_fuse is not None else z
    ws = workspace(x.device)
    if (CONV_TR and spec.R == 3 and spec.S == 3 and spec.stride == 1 and spec.pad == 1
            and spec.C == spec.Cr and spec.C % 64 == 0 and spec.K % 64 == 0):
        # 3x3 tap-reuse kernel (conv_tr.hip): input tile resident in LDS for all nine taps
        r = native().conv_fwd_tr(g, ptr(x), ptr(spec.wc), ptr(bias), ptr(z), ptr(stats), ptr(ws),
                                 ws.numel(), stream_handle(), bn_fuse,
                                 _fin_args(fin, x) if fin is not None else None)
        if r:
            return (z, r == 2) if bn_fuse is not None else z
    if fin is not None:
        _bn_act_fwd_now(fin, fin.fwd_z, x)
    if bn_fuse is not None:
        fused = native().conv_fwd_bn(g, ptr(x), ptr(spec.wc), ptr(bias), ptr(z), ptr(stats),
                                     ptr(ws), ws.numel(), stream_handle(), bn_fuse)
        return z, bool(fused)
    native().conv_fwd(g, ptr(x), ptr(spec.wc), ptr(bias), ptr(z), ptr(stats), ptr(ws), ws.numel(),
                      0, stream_handle())
    return z


class GradLink:
    """Merges the two gradient branches that meet at a residual block's input without an add
    kernel. Both consumers of the tensor (the first conv of the branch and the identity /
    downsample path) report to the link during backward: the first one to run leaves its
    gradient in the link and returns None to autograd; the second one adds its contribution in
    place — a conv dgrad writes ``dx += ...`` from its epilogue — and returns the sum. Autograd's
    own accumulation (None + sum) then needs no kernel. One link serves one forward."""

    def __init__(self, consumers=2):
        self.expected = consumers
        self.seen = 0
        self.buf = None
        self.deferred = None  # (dy, relu_mask): a residual gradient that was never stored
        self.deferred_dgrad = None  # (geom, dz, wc): a strided shortcut's dgrad, run last

    def defer(self, dy, mask):
        """The residual BatchNorm's gradient dres = dy through its ReLU mask, NOT stored: the
        other consumer's accumulating dgrad computes it from (dy, mask) in its epilogue
        (conv_igemm.hip ConvArgs::acc_dy / acc_mask) — one activation-sized write and read
        fewer per identity block."""
        self.seen += 1
        self.deferred = (dy, mask)
        return None

    def offer(self, t):
        """A consumer whose gradient is already a tensor (the BN residual gradient)."""
        self.seen += 1
        if self.buf is None:
            self.buf = t
        else:
            self.buf.add_(t)  # (not hit by the built-in models: the residual producer runs first)
        return self.result()

    def result(self):
        if self.seen < self.expected:
            return None
        out, self.buf = self.buf, None
        return out


# Design switches of the fused paths. Each was measured against the unfused path it replaces
# (profiles cited below) and won on every measured configuration; the unfused paths stay as the
# oracles the GPU tests compare the fused ones against (tests flip these module constants), not
# as run-time options.
#
# 3x3 stride-1 forward convolutions through the tap-reuse kernel (conv_tr.hip); False: the
# implicit-GEMM kernel for every layer
CONV_TR = True
# a block's BatchNorm + ReLU (+ 2x2 pool) forward computed by the NEXT block's tap-reuse conv
# while it loads its input patch (conv_tr.hip fused input; no bn_act_fwd launch); =0 restores the
# separate pass
# (1 = every eligible block, 2 = only blocks without a max-pool: a pooled block's consumer loads
# four pre-pool values per input pixel, measured -1 % at 32 images per GPU but +3 % at 256
# (profiles/r3_fused_bn_input.md))
FUSE_BN_IN = 2
# mode 2 still fuses pooled blocks up to this many images per GPU: at 32 (the 8-GPU share) the
# launch it removes outweighs the 4x patch bytes (b32 0.4132 vs 0.4178 ms; at 64 it loses,
# 0.4933 vs 0.4870; profiles/r3_fused_bn_input.md)
FUSE_BN_IN_POOL_MAX_BATCH = 32
# BatchNorm forward fused into the split-K finish of small conv GEMMs (conv_igemm.hip
# splitk_finish_bnfwd_kernel)
BN_FWD_FUSE = True
# the preceding block's whole BatchNorm backward completed in a small dgrad's split-K finish
# (conv_igemm.hip splitk_finish_bnbwd_kernel; BnBwdFuse chain only)
BN_BWD_APPLY_FUSE = True
# ... and into the classifier head's backward: dx + that BN backward + dW / db in one launch
# (conv_igemm.hip linear_head_bwd_kernel; needs BN_BWD_APPLY_FUSE too)
HEAD_BN_FUSE = True
# ... and its BN + ReLU + 2x2 pool FORWARD folded into the head's forward kernel (linear_ce.hip
# HeadBnIn: one launch fewer; the training loss path only, VGG's 2x2 last block)
HEAD_BN_FWD = True
# residual blocks (BN + residual + ReLU, no pool; ResNet's bn3): the forward stores the ReLU
# mask as one bit per element and the backward reads it instead of the residual tensor, which it
# only ever needed for that mask (bn_act.hip BnArgs::mask; 1/16 of the bytes, twice per layer)
BN_RELU_MASK = True
# ... and an identity block's residual gradient (dy through that mask) is not stored at all: the
# branch's first 1x1 conv rebuilds it in its accumulating dgrad epilogue (GradLink.defer)
RES_DEFER = True
# ... and a projection block's shortcut BatchNorm folded into the block's residual BN passes: the
# downsample conv's PRE-BN output is the residual, normalised inside bn3's apply, and bn3's
# backward reduce / apply also produce the shortcut's dz (bn_act.hip RBN; both BNs see the same
# gradient dy * mask, so they share S1). The shortcut's BN output and its gradient are never
# stored and its own finalize / apply / reduce / finalize / apply launches disappear.
RES_BN_FUSE = True
# ... and a strided shortcut conv whose backward reaches the block input first leaves its dgrad
# to the other branch: that one writes dx, then the shortcut's phase dgrad ACCUMULATES into the
# 1/stride^2 of dx it reaches — no zero fill of dx's untouched phases and no read-back of the
# whole dx by an accumulating second branch (GradLink.deferred_dgrad)
DS_DGRAD_DEFER = True
# largest dgrad output H*W that takes the fused sums: 16 (4x4 / 2x2) at 256 images per GPU,
# 256 (also 16x16 / 8x8) at the strong-scaling shares of at most 128 images (b64 0.4556 vs
# 0.4594 ms, b32 0.3921 vs 0.3952, profiles/r4z3_bn_sums_threshold.md; b128 0.5320 vs 0.5353 on
# the round-6 kernels, every one of 5 in-step trials lower, b256 0.7541 vs 0.7281,
# profiles/r6ae_ab_constants.jsonl); a number here sets one threshold for every batch (tests)
BN_BWD_FUSE_MAX_HW = None


def bn_bwd_fuse_pays(H, W, pool=True, N=None):
    """Fuse the preceding block's BatchNorm-backward sums into this dgrad only when the dgrad
    output is spatially small: H*W <= 16 (VGG's 4x4 / 2x2 layers), or <= 256 at N <= 128 images
    (BN_BWD_FUSE_MAX_HW). Measured (VGG-11, tools/conv_tune.py and the step profiles): on the
    small outputs the fused epilogue costs 2-5 us less than the reduce kernel it replaces; on the
    b256 16x16 / 8x8 outputs its z gather (4 loads per pooled pixel, exposed after the MFMA
    loop) costs more than the streaming reduce pass, at b32..b128 the launch it saves wins.
    Never without a pool (ResNet's conv1 -> conv2 -> conv3 chain): one z load per dgrad output
    element in the epilogue made the big dgrad GEMMs slower than the reduce pass it saves
    (ResNet-50 b256 30.65 vs 28.23 ms, profiles/r2_resnet50_b256.md; again in round 4: 9443 vs
    9573 img/s; the opt-in was removed in round 5)."""
    if not pool:
        return False
    lim = BN_BWD_FUSE_MAX_HW
    if lim is None:
        lim = 256 if N is not None and N <= 128 else 16
    return H * W <= lim


def _masked(dy, mask):
    """dy through ReLU mask bits ([..., C/8] bytes, bit e = channel 8i + e): the stored form of a
    deferred residual gradient (fallback of GradLink.defer)."""
    bits = (mask.unsqueeze(-1).to(torch.int32) >> torch.arange(8, device=mask.device,
                                                               dtype=torch.int32)) & 1
    return torch.where(bits.reshape(dy.shape).bool(), dy, torch.zeros((), dtype=dy.dtype,
                                                                      device=dy.device))


def conv_backward(spec, x, dz, dweight, need_dx, link=None, weight=None, bnf=None, bna=None):
    """dW += wgrad(dz, x); returns dx (or None). Everything is stream-ordered on the current
    stream; with ``weight`` (the parameter whose gradient is dweight) the gradient is announced
    ready here, else by the caller. (A backward side stream for the wgrad was measured slower,
    VGG-11 b256 1.115 vs 1.00 ms: a captured fork/join runs on several hardware queues with a
    completion-signal hop per edge; removed in round 5.)
    ``bna`` = (dz_prev, dgamma_prev, dbeta_prev) pointers (with ``bnf``): the preceding block's
    whole BatchNorm backward may be completed in the dgrad's split-K finish; the return value is
    then (dx, done) — when done, dx was NOT written and dz_prev / dgamma / dbeta were."""
    N, H, W, C = x.shape
    g = spec.geom(N, H, W, weight_krsc(dweight))
    s = stream_handle()
    ws = workspace(x.device)
    if need_dx and link is None and spec.stride == 1 and spec.C == spec.Cr:
        # wgrad + dgrad of this layer as one grouped launch (+ one finish launch) when the
        # kernel policy allows it (conv_igemm.hip ddp_conv_bwd_pair), else the two launches
        dx = torch.empty_like(x)
        done = native().conv_bwd_pair(g, ptr(dz), ptr(spec.wc), ptr(dx), ptr(x), ptr(dweight),
                                      ptr(ws), ws.numel(), s, bn=bnf, bna=bna)
        if weight is not None:
            grad_ready([weight])
        if bnf is not None and len(bnf) > 7:  # input block's sums: 2 = taken in the finish
            return dx, int(done) == 2
        return (dx, int(done) == 1) if bna is not None else dx
    # final: no dgrad of this layer follows, so its finish may apply a registered SGD step
    native().conv_wgrad(g, ptr(dz), ptr(x), ptr(dweight), ptr(ws), ws.numel(), 0, s,
                        final=int(not need_dx))
    if weight is not None:
        grad_ready([weight])
    if not need_dx:
        return (None, False) if (bna is not None or (bnf is not None and len(bnf) > 7)) else None
    if spec.C != spec.Cr:
        raise RuntimeError("dgrad requested for a channel-padded input layer")
    if (DS_DGRAD_DEFER and link is not None and spec.stride > 1 and link.buf is None
            and link.deferred is None and link.deferred_dgrad is None
            and link.seen + 1 < link.expected):
        # strided first branch: its dgrad runs after the other branch wrote dx (accumulating)
        link.deferred_dgrad = (g, dz, spec.wc)
        link.seen += 1
        return None
    if link is not None and link.deferred is not None and spec.stride == 1:
        # second branch onto a deferred first branch: dx = dgrad + dy * mask (dx only written)
        acc_dy, acc_mask = link.deferred
        link.deferred = None
        dx = torch.empty_like(x)
        native().conv_dgrad(g, ptr(dz), ptr(spec.wc), ptr(dx), ptr(ws), ws.numel(), 0, s,
                            accumulate=1, acc_dy=ptr(acc_dy), acc_mask=ptr(acc_mask))
        link.seen += 1
        link.buf = dx
        return link.result()
    if link is not None and link.deferred is not None:  # (not hit: identity blocks are stride 1)
        acc_dy, acc_mask = link.deferred
        link.deferred = None
        link.buf = _masked(acc_dy, acc_mask)
    if link is not None and link.buf is not None:
        # second branch: accumulate into the first branch's gradient from the GEMM epilogue
        native().conv_dgrad(g, ptr(dz), ptr(spec.wc), ptr(link.buf), ptr(ws), ws.numel(), 0, s,
                            accumulate=1)
        link.seen += 1
        return link.result()
    dx = torch.empty_like(x)
    l0_mode = bnf is not None and len(bnf) > 7  # (input block's sums: pair launch only)
    done = native().conv_dgrad(g, ptr(dz), ptr(spec.wc), ptr(dx), ptr(ws), ws.numel(), 0, s,
                               bn=None if l0_mode else bnf, bna=bna)
    if link is not None and link.deferred_dgrad is not None:
        gd, dzd, wcd = link.deferred_dgrad
        link.deferred_dgrad = None
        native().conv_dgrad(gd, ptr(dzd), ptr(wcd), ptr(dx), ptr(ws), ws.numel(), 0, s,
                            accumulate=1)
    if link is not None:
        link.seen += 1
        link.buf = dx
        return link.result()
    if l0_mode:
        return dx, False
    return (dx, bool(done)) if bna is not None else dx


# VGG input block (conv 3x3 over the 8-channel padded image -> 64, BN, ReLU, 2x2 pool) through
# conv_l0.hip: its pre-BN activation z (the network's largest tensor) is recomputed from the
# input in every pass that needs it instead of being stored and streamed four times.
# False: conv_smallk + bn_act passes.
L0_FUSE = True
# ... and its BN-backward sums taken in the next block's dgrad split-K finish when that dgrad has
# one (conv_igemm.hip BnBwdFuse::code; else l0_sums_kernel). False: always the separate pass.
# Up to L0_SUMS_IN_FINISH_MAX_BATCH images per GPU: at b64 0.4312 vs 0.4336 ms, at b128 the
# separate pass wins (0.5290 vs 0.5333; in-step A/B, every trial: profiles/r6af_ab_constants.jsonl)
L0_SUMS_IN_FINISH = True
L0_SUMS_IN_FINISH_MAX_BATCH = 64


def l0_serves(spec, x):
    N, H, W, C = x.shape
    if not (L0_FUSE and x.is_cuda and C == 8 and spec.C == 8 and spec.K == 64 and spec.pool
            and spec.relu and not spec.maxpool3 and not spec.residual):
        return False
    cache = spec.__dict__.setdefault("_l0_cache", {})
    if (N, H, W) not in cache:
        cache[(N, H, W)] = bool(native().l0_ok(spec.geom(N, H, W)))
    return cache[(N, H, W)]


def _defer_bn(spec, residual, running_mean, N, Ho, Wo):
    """Defer this block's BatchNorm + ReLU (+ pool) forward into the next block's conv: only on
    a plain Conv->BN->ReLU(->pool) chain (no residual, batch statistics) whose next conv the
    tap-reuse kernel serves with a fused input (conv_tr.hip)."""
    nxt = spec.next
    if (not FUSE_BN_IN or not CONV_TR or nxt is None or residual is not None
            or running_mean is not None or nxt.C != spec.K or nxt.Cr != nxt.C
            or nxt.R != 3 or nxt.stride != 1 or nxt.pad != 1):
        return False
    if FUSE_BN_IN == 2 and spec.pool and N > FUSE_BN_IN_POOL_MAX_BATCH:
        return False
    if spec.pool and (Ho * 2 != spec._out_p or Wo * 2 != spec._out_q):
        return False
    g = nxt.geom(N, Ho, Wo)
    return bool(native().conv_tr_would_serve(g, workspace(nxt.wc.device).numel(),
                                             2 if spec.pool else 1))


class _ConvPreBNFn(torch.autograd.Function):
    """A projection shortcut's conv whose BatchNorm runs inside its consumer's residual BN
    passes (RES_BN_FUSE): z = conv(x) + bias, with z's batch statistics from the GEMM epilogue.
    The consumer normalises z with this spec's table and its backward hands autograd dz — the
    gradient at z — with this BN's gamma / beta gradients already accumulated and announced."""

    @staticmethod
    def forward(ctx, x, weight, bias, spec, in_link=None):
        spec.maybe_pack()
        spec.dz_fused = None
        spec.deferred = None
        z = conv_forward(spec, x, bias, spec.stats)
        spec.fwd_z = None
        ctx.spec, ctx.in_link = spec, in_link
        ctx.save_for_backward(x, weight, bias)
        return z

    @staticmethod
    def backward(ctx, dz):
        x, weight, bias = ctx.saved_tensors
        if bias is not None:
            ensure_grad(bias)  # analytically zero under batch-statistics BN (bn_act.hip)
            grad_ready([bias])
        dx = conv_backward(ctx.spec, x, dz.contiguous(), ensure_grad(weight),
                           ctx.needs_input_grad[0], ctx.in_link, weight=weight)
        return dx, None, None, None, None


def conv_pre_bn(x, spec, in_link=None):
    """The conv of ``spec`` with its BatchNorm left to the residual block that consumes it
    (``conv_bn_act(..., residual=z, res_bn=spec)``)."""
    conv = spec.conv
    return _ConvPreBNFn.apply(x, conv.weight, conv.bias, spec, in_link)


def res_bn_fuse_ok(spec):
    """The residual BN of ``spec`` can take a projection shortcut's BatchNorm (bn_act.hip
    res_shape_ok; the backward needs the ReLU mask bits)."""
    return (RES_BN_FUSE and BN_RELU_MASK and spec.residual and spec.relu and not spec.pool
            and spec.K % 8 == 0 and 256 % (spec.K // 8) == 0)


class _ConvBNActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, gamma, beta, residual, spec, in_link=None, res_link=None,
                res_bn=None):
        spec.maybe_pack()
        spec.dz_fused = None  # a fused BN backward of an earlier pass must never be consumed
        spec.deferred = None
        # the preceding block deferred its BatchNorm forward into this conv (x = its unwritten
        # output; a pipelined step's cut passes a detached view of the same storage)
        prev = spec.prev
        fin = None
        if prev is not None and prev.deferred is not None:
            if prev.deferred.data_ptr() == x.data_ptr():
                fin = prev
            else:  # not consumed by this block: materialise it where it is
                _bn_act_fwd_now(prev, prev.fwd_z, prev.deferred)
            prev.deferred = None
        N, H, W, _ = x.shape
        stats = spec.stats  # zeroed by the model's per-forward StepScratch.zero()
        P, Q = spec.out_hw(H, W)
        Ho, Wo = (P // 2, Q // 2) if spec.pool else (P, Q)
        if spec.maxpool3:
            if spec.pool or residual is not None:
                raise ValueError("the fused 3x3 max-pool excludes the 2x2 pool and a residual")
            Ho, Wo = (P - 1) // 2 + 1, (Q - 1) // 2 + 1
        spec._out_p, spec._out_q = P, Q
        y = torch.empty(N, Ho, Wo, spec.K, dtype=BF16, device=x.device)
        if residual is not None:
            check(residual, BF16, (N, P, Q, spec.K), "residual")
        if res_bn is not None and (residual is None or res_link is not None
                                   or not res_bn_fuse_ok(spec) or res_bn.K != spec.K):
            raise ValueError("shortcut BatchNorm fold: residual block with ReLU mask only")
        ctx.res_bn = res_bn
        bn = spec.bn
        rm = rv = None
        use_running = 0
        if bn.track_running_stats and bn.running_mean is not None:
            rm, rv = bn.running_mean, bn.running_var
            use_running = 0 if bn.training else 1
        ctx.l0 = residual is None and rm is None and fin is None and l0_serves(spec, x)
        if ctx.l0:
            # input block: statistics pass + BN/ReLU/pool pass, z never stored (conv_l0.hip)
            # code: per pooled value, the window position its gradient goes to (1 B each)
            # and that pixel's z (bf16), so the backward sums need no conv
            code = torch.empty(N, Ho, Wo, spec.K, dtype=torch.uint8, device=x.device)
            zw = torch.empty(N, Ho, Wo, spec.K, dtype=BF16, device=x.device)
            native().l0_fwd(spec.geom(N, H, W), ptr(x), ptr(spec.wc), ptr(bias), spec.eps,
                            int(spec.relu), ptr(stats), ptr(gamma), ptr(beta), ptr(spec.coef),
                            ptr(y), ptr(code), ptr(zw), stream_handle())
            ctx.l0_code = (code, zw)
            spec.l0_code = (code, zw)  # (the next block's dgrad finish may take the sums)
            spec.l0_sums_ready = False
            spec.fwd_z = None
            spec.last_deferred = False
            ctx.pool3_idx = None
            ctx.spec, ctx.has_res, ctx.in_link, ctx.res_link = spec, False, in_link, res_link
            ctx.prev_z = None
            ctx.save_for_backward(x, None, stats, weight, bias, gamma, beta, None)
            return y
        fused = False
        if residual is None and rm is None and BN_FWD_FUSE:
            # batch-statistics BN without residual (VGG): may run inside the conv's split-K finish
            z, fused = conv_forward(spec, x, bias, stats,
                                    bn_fuse=(ptr(gamma), ptr(beta), spec.eps, int(spec.relu),
                                             int(spec.pool), ptr(spec.coef), ptr(y), P, Q),
                                    fin=fin)
        else:
            z = conv_forward(spec, x, bias, stats, fin=fin)
        spec.fwd_z = z
        ctx.pool3_idx = None
        # the classifier head computes this block's BN + ReLU + pool (set by forward_loss on the
        # last block; linear_ce.hip HeadBnIn) — or the next conv does (conv_tr fused input)
        to_head = (HEAD_BN_FWD and getattr(spec, "defer_to_head", False) and residual is None
                   and rm is None and spec.pool and P == 2 and Q == 2 and spec.relu)
        spec.last_deferred = (not fused and not spec.maxpool3
                              and (to_head or _defer_bn(spec, residual, rm, N, Ho, Wo)))
        if spec.maxpool3:
            idx = torch.empty(N, Ho, Wo, spec.K, dtype=torch.uint8, device=x.device)
            native().bn_pool3_fwd(N, P, Q, spec.K, int(spec.relu), spec.eps, ptr(z), ptr(stats),
                                  ptr(gamma), ptr(beta), ptr(y), ptr(idx), stream_handle(),
                                  ptr(rm), ptr(rv),
                                  float(bn.momentum if bn.momentum is not None else 0.1),
                                  use_running, ptr(spec.coef))
            ctx.pool3_idx = idx
        elif spec.last_deferred:
            spec.deferred = y  # computed by the next block's conv or the head (see to_head)
        elif not fused:
            mask = None
            if (BN_RELU_MASK and residual is not None and spec.relu and not spec.pool
                    and any(ctx.needs_input_grad) and spec.K % 8 == 0):
                mask = torch.empty(N, P, Q, spec.K // 8, dtype=torch.uint8, device=x.device)
            ctx.relu_mask = mask
            rk = {}
            if res_bn is not None:  # residual = the shortcut's pre-BN z, normalised here
                rb = res_bn.bn
                rk = dict(rstats=ptr(res_bn.stats), rgamma=ptr(rb.weight), rbeta=ptr(rb.bias),
                          rcoef=ptr(res_bn.coef), rrunning_mean=ptr(rb.running_mean),
                          rrunning_var=ptr(rb.running_var), reps=res_bn.eps,
                          rmomentum=float(rb.momentum if rb.momentum is not None else 0.1))
            native().bn_act_fwd(N, P, Q, spec.K, int(spec.pool), int(spec.relu), spec.eps, ptr(z),
                                ptr(residual), ptr(stats), ptr(gamma), ptr(beta), ptr(y),
                                stream_handle(), ptr(rm), ptr(rv),
                                float(bn.momentum if bn.momentum is not None else 0.1),
                                use_running, ptr(spec.coef), mask=ptr(mask), **rk)
        ctx.spec = spec
        ctx.has_res = residual is not None
        ctx.in_link, ctx.res_link = in_link, res_link
        # the preceding block's conv output of THIS forward (for the fused BN-backward sums)
        ctx.prev_z = spec.prev.fwd_z if spec.prev is not None else None
        ctx.save_for_backward(x, z, stats, weight, bias, gamma, beta, residual)
        return y

    @staticmethod
    def backward(ctx, dy):
        spec = ctx.spec
        x, z, stats, weight, bias, gamma, beta, residual = ctx.saved_tensors
        if ctx.l0:
            # input block: BN-backward sums + dz passes over the recomputed z, then the weight
            # gradient GEMM on dz (the input itself needs no gradient)
            N, H, W, _ = x.shape
            dy = dy.contiguous()
            gw, gg, gbt = ensure_grad(weight), ensure_grad(gamma), ensure_grad(beta)
            if bias is not None:
                ensure_grad(bias)  # analytically zero under batch-statistics BN (bn_act.hip)
            dz = torch.empty(N, H, W, spec.K, dtype=BF16, device=x.device)
            ready, spec.l0_sums_ready = getattr(spec, "l0_sums_ready", False), False
            native().l0_bwd(spec.geom(N, H, W), ptr(x), ptr(spec.wc), ptr(bias), spec.eps,
                            int(spec.relu), ptr(spec.coef), ptr(dy), ptr(spec.sums), ptr(dz),
                            ptr(gg), ptr(gbt), ptr(ctx.l0_code[0]), ptr(ctx.l0_code[1]),
                            stream_handle(), sums_ready=int(ready))
            ctx.l0_code = None
            spec.l0_code = None
            grad_ready([gamma, beta, bias])
            dx = conv_backward(spec, x, dz, gw, ctx.needs_input_grad[0], ctx.in_link,
                               weight=weight)
            return dx, None, None, None, None, None, None, None, None, None
        N, P, Q, K = z.shape
        sums = spec.sums  # zeroed together with the statistics at the start of the forward
        mask = getattr(ctx, "relu_mask", None)
        ctx.relu_mask = None
        # identity block: the residual gradient goes to the branch's first conv, whose
        # accumulating dgrad can rebuild it from (dy, mask) — never store it (RES_DEFER)
        defer = (RES_DEFER and mask is not None and ctx.res_link is not None
                 and ctx.needs_input_grad[5] and ctx.res_link.seen == 0
                 and ctx.res_link.buf is None)
        dres = torch.empty_like(z) if (ctx.has_res and ctx.needs_input_grad[5]
                                       and not defer) else None
        gw = ensure_grad(weight)
        gb = ensure_grad(bias) if bias is not None else None
        gg = ensure_grad(gamma)
        gbt = ensure_grad(beta)
        sums_ready, spec.sums_ready = spec.sums_ready, False
        dz_done, spec.dz_fused = spec.dz_fused, None
        spec.fwd_z = None
        if dz_done is not None:
            # the next block's dgrad finish already ran this block's whole BN backward (dz,
            # dgamma, dbeta; conv_igemm.hip splitk_finish_bnbwd_kernel): dy was never written
            dz, zref = dz_done
            if zref is None or zref.data_ptr() != z.data_ptr():
                raise RuntimeError("fused BatchNorm backward belongs to another forward pass "
                                   "(stale dz_fused): refusing to use an unwritten gradient")
        elif ctx.pool3_idx is not None:  # stem: pooled gradient routed by the window argmax
            dy = dy.contiguous()
            dz = torch.empty_like(z)
            native().bn_pool3_bwd(N, P, Q, K, int(spec.relu), spec.eps, ptr(z), ptr(dy),
                                  ptr(ctx.pool3_idx), ptr(sums), ptr(dz), ptr(gg), ptr(gbt),
                                  stream_handle(), ptr(spec.coef))
            ctx.pool3_idx = None
        elif ctx.res_bn is not None:
            # + the projection shortcut's BN backward: dres = the gradient at ITS conv output
            rs, rb = ctx.res_bn, ctx.res_bn.bn
            ctx.res_bn = None
            if mask is None or sums_ready or dz_done is not None:
                raise RuntimeError("shortcut BatchNorm fold needs the forward's ReLU mask")
            dy = dy.contiguous()
            dz = torch.empty_like(z)
            if dres is None:
                dres = torch.empty_like(z)
            rg, rbt = ensure_grad(rb.weight), ensure_grad(rb.bias)
            native().bn_act_bwd(N, P, Q, K, int(spec.pool), int(spec.relu), spec.eps, ptr(z),
                                ptr(residual), ptr(stats), ptr(gamma), ptr(beta), ptr(dy),
                                ptr(sums), ptr(dz), 0, ptr(gg), ptr(gbt), ptr(gb),
                                stream_handle(), ptr(spec.coef), mask=ptr(mask),
                                rcoef=ptr(rs.coef), rsums=ptr(rs.sums), rdz=ptr(dres),
                                rdgamma=ptr(rg), rdbeta=ptr(rbt))
            grad_ready([rb.weight, rb.bias])
        else:
            dy = dy.contiguous()
            dz = torch.empty_like(z)
            native().bn_act_bwd(N, P, Q, K, int(spec.pool), int(spec.relu), spec.eps, ptr(z),
                                0 if mask is not None else ptr(residual), ptr(stats), ptr(gamma),
                                ptr(beta), ptr(dy), ptr(sums), ptr(dz), ptr(dres), ptr(gg),
                                ptr(gbt), ptr(gb), stream_handle(), ptr(spec.coef),
                                sums_ready=int(sums_ready), mask=ptr(mask))
        grad_ready([gamma, beta, bias])
        if defer:
            dres = ctx.res_link.defer(dy, mask)
        elif ctx.res_link is not None and dres is not None:
            dres = ctx.res_link.offer(dres)
        bnf = bna = None
        prev = spec.prev
        if (_common.BN_BWD_FUSE and prev is not None and ctx.prev_z is not None
                and ctx.needs_input_grad[0] and ctx.in_link is None and spec.stride == 1
                and not prev.residual and prev.K == spec.C and spec.C == spec.Cr
                and bn_bwd_fuse_pays(x.shape[1], x.shape[2], prev.pool, x.shape[0])):
            pz = ctx.prev_z
            bnf = (ptr(pz), ptr(prev.coef), ptr(prev.sums), int(prev.pool), int(prev.relu),
                   pz.shape[1], pz.shape[2])
            if BN_BWD_APPLY_FUSE:
                dz_prev = torch.empty_like(pz)
                bna = (ptr(dz_prev), ptr(ensure_grad(prev.bn.weight)),
                       ptr(ensure_grad(prev.bn.bias)))
        l0c = getattr(prev, "l0_code", None) if prev is not None else None
        if (bnf is None and L0_SUMS_IN_FINISH and l0c is not None and ctx.needs_input_grad[0]
                and x.shape[0] <= L0_SUMS_IN_FINISH_MAX_BATCH
                and ctx.in_link is None and spec.stride == 1 and prev.K == spec.C
                and spec.C == spec.Cr and x.shape[1] * 2 == prev._out_p):
            # the input block's BN-backward sums in this dgrad's split-K finish (conv_l0.hip's
            # recorded window codes + winner z): its backward skips l0_sums_kernel
            code, zw = l0c
            bl0 = (ptr(zw), ptr(prev.coef), ptr(prev.sums), 1, int(prev.relu), x.shape[1],
                   x.shape[2], ptr(code))
            dx, taken = conv_backward(spec, x, dz, gw, True, None, weight=weight, bnf=bl0)
            prev.l0_sums_ready = bool(taken)
        elif bna is not None:
            dx, done = conv_backward(spec, x, dz, gw, ctx.needs_input_grad[0], ctx.in_link,
                                     weight=weight, bnf=bnf, bna=bna)
            if done:  # prev's backward skips its BN backward; dx was not written
                prev.dz_fused = (dz_prev, ctx.prev_z)
            else:
                prev.sums_ready = True
        else:
            if bnf is not None:
                prev.sums_ready = True
            dx = conv_backward(spec, x, dz, gw, ctx.needs_input_grad[0], ctx.in_link,
                               weight=weight, bnf=bnf)
        ctx.prev_z = None
        return dx, None, None, None, None, dres, None, None, None, None


def conv_bn_act(x, spec, residual=None, in_link=None, res_link=None, res_bn=None):
    """Fused conv -> BN (+residual) -> ReLU (-> 2x2 pool). ``in_link`` / ``res_link``: GradLink
    through which the input / residual gradient is merged with the other branch (ResNet).
    ``res_bn``: the spec whose BatchNorm normalises ``residual`` here (its conv_pre_bn output)."""
    conv, bn = spec.conv, spec.bn
    return _ConvBNActFn.apply(x, conv.weight, conv.bias, bn.weight, bn.bias, residual, spec,
                              in_link, res_link, res_bn)


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


class _LinearCEFn(torch.autograd.Function):
    """Classifier head fused with the mean softmax cross-entropy: ONE kernel computes the logits,
    the loss and dlogits = (softmax - onehot) / B; the backward consumes dlogits scaled by the
    incoming scalar gradient through a device pointer (no elementwise kernel). ``acc``
    optionally receives a running sum of the loss across steps (TrainStep's meter) from the
    same kernel."""

    @staticmethod
    def forward(ctx, x, weight, bias, labels, acc, transient, bn_prev=None):
        B, F = x.shape
        # the Conv->BN->ReLU->pool block whose output x is: its BN backward may be fused into
        # the head's backward (conv_igemm.hip linear_head_bwd_kernel)
        ctx.bn_prev = bn_prev
        ctx.prev_z = bn_prev.fwd_z if bn_prev is not None else None
        J = weight.shape[0]
        check(x, BF16, name="linear input")
        labels = labels.to(torch.int64).contiguous()
        loss = (step_scratch(x.device).take_transient(1).view(()) if transient
                else torch.zeros((), dtype=F32, device=x.device))
        dl = torch.empty(B, J, dtype=F32, device=x.device)
        if (bn_prev is not None and bn_prev.deferred is not None
                and bn_prev.deferred.data_ptr() == x.data_ptr() and ctx.prev_z is not None):
            # the last block deferred its BN + ReLU + pool here: x is written by this kernel
            bn_prev.deferred = None
            bn = bn_prev.bn
            native().bn_pool_linear_ce_fwd(ptr(ctx.prev_z), ptr(bn_prev.stats), ptr(bn.weight),
                                           ptr(bn.bias), bn_prev.eps, int(bn_prev.relu),
                                           ptr(bn_prev.coef), ptr(x), ptr(weight), ptr(bias),
                                           ptr(labels), B, F, J, ptr(dl), ptr(loss),
                                           stream_handle(), loss_acc=ptr(acc))
        else:
            native().linear_ce_fwd(ptr(x), ptr(weight), ptr(bias), ptr(labels), B, F, J, 0,
                                   ptr(dl), ptr(loss), 0, stream_handle(), loss_acc=ptr(acc))
        ctx.save_for_backward(x, weight, bias, dl)
        return loss

    @staticmethod
    def backward(ctx, g):
        x, weight, bias, dl = ctx.saved_tensors
        B, F = x.shape
        J = weight.shape[0]
        g = g.contiguous().float()
        gw = ensure_grad(weight)
        gb = ensure_grad(bias) if bias is not None else None
        prev, pz = ctx.bn_prev, ctx.prev_z
        ctx.prev_z = None
        if (prev is not None and pz is not None and ctx.needs_input_grad[0] and BN_BWD_APPLY_FUSE
                and HEAD_BN_FUSE
                and _common.BN_BWD_FUSE and prev.pool and not prev.residual
                and pz.shape[1] == 2 and pz.shape[2] == 2 and prev.K == F):
            dz_prev = torch.empty_like(pz)
            bnf = (ptr(pz), ptr(prev.coef), ptr(prev.sums), 1, int(prev.relu), 2, 2)
            bna = (ptr(dz_prev), ptr(ensure_grad(prev.bn.weight)), ptr(ensure_grad(prev.bn.bias)))
            # dx + the block's whole BN backward + dW / db: one launch (linear_head_bwd_kernel)
            done = native().linear_head_bwd_bn(ptr(dl), ptr(weight), ptr(x), B, F, J, ptr(g),
                                               bnf, bna, ptr(gw), ptr(gb), stream_handle())
            if done:  # dx never materialised: the block's backward takes dz_prev
                prev.dz_fused = (dz_prev, pz)
                grad_ready([weight, bias])
                return torch.empty_like(x), None, None, None, None, None, None
        dx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        native().linear_bwd(ptr(dl), ptr(x), ptr(weight), B, F, J, ptr(g), ptr(dx), ptr(gw),
                            ptr(gb), stream_handle())
        grad_ready([weight, bias])
        return dx, None, None, None, None, None, None


def linear_cross_entropy(x, linear, labels, acc=None, transient=False, bn_prev=None):
    """mean CE(linear(x), labels) in one kernel (J <= 16); see _LinearCEFn. ``transient=True``
    returns the loss in the per-forward scratch (saves a fill launch; valid until the next
    model forward on this device — the captured training step uses it)."""
    if linear.weight.shape[0] > 16:
        raise ValueError("linear_cross_entropy supports at most 16 outputs")
    return _LinearCEFn.apply(x, linear.weight, linear.bias, labels, acc, transient, bn_prev)


def linear_small(x, linear):
    if linear.weight.shape[0] > 16:
        raise ValueError("linear_small supports at most 16 outputs")
    return _LinearSmallFn.apply(x, linear.weight, linear.bias)


class _CrossEntropyFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels):
        B, J = logits.shape
        logits = logits.contiguous()
        if logits.dtype not in (F32, BF16):
            raise ValueError("logits must be fp32 or bf16")
        is_bf16 = int(logits.dtype == BF16)
        labels = labels.to(torch.int64).contiguous()
        loss = torch.zeros((), dtype=F32, device=logits.device)
        dl = torch.empty(B, J, dtype=logits.dtype, device=logits.device)  # dlogits in logits dtype
        native().softmax_ce(ptr(logits), is_bf16, ptr(labels), B, J, ptr(loss), 0, ptr(dl),
                            is_bf16, stream_handle())
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


# ------------------------------------------------------------------ ResNet building blocks
class _MaxPoolFn(torch.autograd.Function):
    """MaxPool2d(k, stride, padding) on NHWC bf16 with a 1-byte argmax per output element."""

    @staticmethod
    def forward(ctx, x, k, stride, pad):
        check(x, BF16, name="maxpool input")
        N, H, W, C = x.shape
        Ho = (H + 2 * pad - k) // stride + 1
        Wo = (W + 2 * pad - k) // stride + 1
        y = torch.empty(N, Ho, Wo, C, dtype=BF16, device=x.device)
        idx = torch.empty(N, Ho, Wo, C, dtype=torch.uint8, device=x.device)
        native().maxpool_fwd(ptr(x), N, H, W, C, k, k, stride, pad, Ho, Wo, ptr(y), ptr(idx),
                             stream_handle())
        ctx.save_for_backward(idx)
        ctx.cfg = (N, H, W, C, k, stride, pad, Ho, Wo)
        return y

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        N, H, W, C, k, stride, pad, Ho, Wo = ctx.cfg
        dy = dy.contiguous()
        dx = torch.empty(N, H, W, C, dtype=BF16, device=dy.device)
        native().maxpool_bwd(ptr(dy), ptr(idx), N, H, W, C, k, k, stride, pad, Ho, Wo, ptr(dx),
                             stream_handle())
        return dx, None, None, None


def max_pool(x, k=3, stride=2, pad=1):
    return _MaxPoolFn.apply(x, k, stride, pad)


class _GlobalAvgPoolFn(torch.autograd.Function):
    """AdaptiveAvgPool2d(1) + flatten: NHWC bf16 [N, H, W, C] -> [N, C]."""

    @staticmethod
    def forward(ctx, x):
        check(x, BF16, name="avgpool input")
        N, H, W, C = x.shape
        y = torch.empty(N, C, dtype=BF16, device=x.device)
        native().avgpool_fwd(ptr(x), N, H * W, C, ptr(y), stream_handle())
        ctx.cfg = (N, H, W, C)
        return y

    @staticmethod
    def backward(ctx, dy):
        N, H, W, C = ctx.cfg
        dx = torch.empty(N, H, W, C, dtype=BF16, device=dy.device)
        native().avgpool_bwd(ptr(dy.contiguous()), N, H * W, C, ptr(dx), stream_handle())
        return dx


def global_avg_pool(x):
    return _GlobalAvgPoolFn.apply(x)


class LinearGemmSpec(ConvBNActSpec):
    """nn.Linear(F, J) run as a 1x1 convolution on the MFMA implicit-GEMM kernels
    (weight [J][F] is exactly a [J][F][1][1] conv weight; J and F multiples of 8)."""

    def __init__(self, linear):  # noqa: super().__init__ is not used (no BN, 2-D weight)
        J, F = linear.weight.shape
        if J % 8 or F % 8:
            raise ValueError("GEMM linear needs in/out features divisible by 8")
        self.linear = linear
        self.conv, self.bn = linear, None
        self.K, self.Cr, self.R, self.S, self.C = J, F, 1, 1, F
        self.stride, self.pad = 1, 0
        self.relu, self.pool, self.residual = False, False, False
        self.eps = 1e-5
        dev = linear.weight.device
        self.wc = torch.empty(J, F, dtype=BF16, device=dev)
        self.wt = None
        self._packed_version = None
        linear.weight._ddp_amd_pack = self.pack_desc
        self.stats = None
        self.sums = None


class _LinearGemmFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, spec):
        spec.maybe_pack()
        B, F = x.shape
        check(x, BF16, name="linear input")
        x4 = x.view(B, 1, 1, F)
        y = conv_forward(spec, x4, bias, None)
        ctx.spec = spec
        ctx.save_for_backward(x4, weight, bias)
        return y.view(B, spec.K)

    @staticmethod
    def backward(ctx, dy):
        spec = ctx.spec
        x4, weight, bias = ctx.saved_tensors
        B = x4.shape[0]
        dy = dy.contiguous().to(BF16)
        gw = ensure_grad(weight)
        if bias is not None:
            native().colsum(ptr(dy), B, spec.K, ptr(ensure_grad(bias)), stream_handle())
        dx = conv_backward(spec, x4, dy.view(B, 1, 1, spec.K), gw, ctx.needs_input_grad[0])
        grad_ready([weight, bias])
        return (dx.view(B, -1) if dx is not None else None), None, None, None


def linear_gemm(x, spec):
    lin = spec.linear
    return _LinearGemmFn.apply(x, lin.weight, lin.bias, spec)
