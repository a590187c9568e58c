"""ResNet-50 (driver config) on the gfx950 path vs the CPU fp32 ATen oracle."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def _bf16_emulated_logits_err(model, x, ref):
    m = copy.deepcopy(model)
    rb = lambda t: t.to(torch.bfloat16).float()  # noqa: E731
    for mod in m.modules():
        if isinstance(mod, (torch.nn.Conv2d, torch.nn.Linear, torch.nn.BatchNorm2d)):
            if not isinstance(mod, torch.nn.BatchNorm2d):
                mod.weight.data = rb(mod.weight.data)
            mod.register_forward_pre_hook(lambda mm, inp: (rb(inp[0]),))
            mod.register_forward_hook(lambda mm, inp, o: rb(o))
    with torch.no_grad():
        out = m(x)
    return float((out - ref).norm() / ref.norm())


def test_resnet50_train_step_matches_cpu(native_ext):
    from ddp_amd.models.resnet import resnet50
    from ddp_amd.engine import CrossEntropyLoss
    from ddp_amd.optim import FusedSGD
    torch.manual_seed(0)
    cpu = resnet50(num_classes=16)
    gpu = copy.deepcopy(cpu).cuda()
    opt = FusedSGD(gpu.parameters(), lr=0.1)
    # 16 x 128 x 128: layer4 BN statistics over 16 x 4 x 4 values (8 x 2 x 2 is too noisy)
    x = torch.randn(16, 3, 128, 128).to(torch.bfloat16).float()
    y = torch.randint(0, 16, (16,))
    crit = CrossEntropyLoss()
    out_c = cpu(x)
    lc = crit(out_c, y)
    lc.backward()
    opt.zero_grad()
    out = gpu(x.cuda())
    assert out.shape == (16, 16)
    # forward error is at the level of bf16 rounding itself: an fp32 CPU model that rounds every
    # conv/linear/BN input, output and weight to bf16 lands ~0.12 away from fp32 on this net
    ref_err = _bf16_emulated_logits_err(cpu, x, out_c.detach())
    gpu_err = float((out.float().cpu() - out_c.detach()).norm() / out_c.detach().norm())
    print("logits rel err: gpu", gpu_err, "bf16-emulated cpu", ref_err)
    assert gpu_err < 1.5 * ref_err + 0.01
    lg = crit(out, y.cuda())
    lg.backward()
    torch.cuda.synchronize()
    assert abs(float(lg) - float(lc)) < 0.05 * max(1.0, abs(float(lc)))
    # running statistics were updated like torch's BatchNorm
    assert torch.allclose(gpu.bn1.running_mean.cpu(), cpu.bn1.running_mean, rtol=0.05, atol=1e-3)
    assert int(gpu.bn1.num_batches_tracked) == 1
    cos = {}
    for (n, pc), pg in zip(cpu.named_parameters(), gpu.parameters()):
        a, b = pg.grad.cpu().reshape(-1), pc.grad.reshape(-1)
        if b.norm() == 0:
            continue
        cos[n] = float(torch.dot(a, b) / (a.norm() * b.norm() + 1e-20))
    print({k: round(v, 3) for k, v in list(cos.items())[:12]})
    # The WHOLE random-init ResNet-50 backward is ill-conditioned: in pure fp32 on the CPU, a
    # 2^-9 relative perturbation of the input alone drops the cosine of conv1.weight's gradient
    # to ~0.46 (fc.weight stays ~0.998, layer4.2.bn3 ~0.98) — max-pool routing and ReLU masks
    # flip. So only the late-layer gradients are compared here; per-block correctness is pinned
    # by test_bottleneck_block_matches_cpu (cosine > 0.97 on every parameter).
    assert cos["fc.weight"] > 0.97 and cos["fc.bias"] > 0.99
    assert cos["layer4.2.bn3.weight"] > 0.9
    # eval mode uses running statistics
    gpu.eval()
    cpu.eval()
    with torch.no_grad():
        oe_g, oe_c = gpu(x.cuda()).float().cpu(), cpu(x)
    assert float((oe_g - oe_c).norm() / oe_c.norm()) < 0.1


def test_linear_gemm_and_bf16_ce(native_ext):
    import torch.nn.functional as F
    from ddp_amd.ops.layers import LinearGemmSpec, linear_gemm, cross_entropy
    torch.manual_seed(0)
    lin = torch.nn.Linear(256, 1000).cuda()
    lin.weight.grad = torch.zeros_like(lin.weight)
    lin.bias.grad = torch.zeros_like(lin.bias)
    spec = LinearGemmSpec(lin)
    x = torch.randn(32, 256, device="cuda").to(torch.bfloat16).requires_grad_(True)
    y = torch.randint(0, 1000, (32,), device="cuda")
    logits = linear_gemm(x, spec)
    loss = cross_entropy(logits, y)
    loss.backward()
    xr = x.detach().float().requires_grad_(True)
    wr = lin.weight.detach().clone().requires_grad_(True)
    br = lin.bias.detach().clone().requires_grad_(True)
    lr_ = F.linear(xr, wr, br)
    ref = F.cross_entropy(lr_, y)
    ref.backward()

    def rel(a, b):
        return float((a.float() - b.float()).norm() / b.float().norm())
    assert rel(logits, lr_) < 1e-2
    assert abs(float(loss) - float(ref)) < 2e-2
    assert rel(x.grad, xr.grad) < 3e-2
    assert rel(lin.weight.grad, wr.grad) < 3e-2
    assert rel(lin.bias.grad, br.grad) < 3e-2


def test_bottleneck_block_matches_cpu(native_ext):
    """One stride-2 bottleneck with downsample (no max-pool routing): well conditioned."""
    from ddp_amd.models.resnet import Bottleneck
    from ddp_amd.optim import FusedSGD
    from ddp_amd.ops.layers import global_avg_pool
    torch.manual_seed(0)
    ds = torch.nn.Sequential(torch.nn.Conv2d(64, 256, 1, stride=2, bias=False),
                             torch.nn.BatchNorm2d(256))
    cpu = Bottleneck(64, 64, stride=2, downsample=ds)
    gpu = copy.deepcopy(cpu).cuda()
    FusedSGD(gpu.parameters(), lr=0.1).zero_grad()
    x = torch.randn(8, 64, 16, 16).to(torch.bfloat16).float()
    w = torch.randn(8, 256)
    out_c = (cpu(x).mean((2, 3)) * w).sum()
    out_c.backward()
    xn = x.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16).cuda()
    h = gpu.forward_fused(xn)
    out_g = (global_avg_pool(h).float() * w.cuda()).sum()
    out_g.backward()
    torch.cuda.synchronize()
    assert abs(float(out_g) - float(out_c)) < 0.05 * max(1.0, abs(float(out_c)))
    cos = {}
    for (n, pc), pg in zip(cpu.named_parameters(), gpu.parameters()):
        a, b = pg.grad.cpu().reshape(-1), pc.grad.reshape(-1)
        cos[n] = float(torch.dot(a, b) / (a.norm() * b.norm() + 1e-20))
    print(cos)
    assert min(cos.values()) > 0.97, cos


def test_bottleneck_shortcut_bn_fold_matches_unfolded(native_ext):
    """The projection shortcut's BatchNorm folded into the block's residual BN passes
    (ops/layers.py RES_BN_FUSE, bn_act.hip RBN) gives the unfolded block's output, input
    gradient and parameter gradients (both BNs' gamma / beta, the shortcut conv) and the same
    running statistics — up to the one rounding it removes (the shortcut BN output is not
    stored as bf16) and the atomics order."""
    from ddp_amd.models.resnet import Bottleneck
    from ddp_amd.optim import FusedSGD
    from ddp_amd.ops import layers
    from ddp_amd.ops.layers import global_avg_pool
    torch.manual_seed(1)
    ds = torch.nn.Sequential(torch.nn.Conv2d(128, 512, 1, stride=2, bias=False),
                             torch.nn.BatchNorm2d(512))
    base = Bottleneck(128, 128, stride=2, downsample=ds)
    x = torch.randn(16, 28, 28, 128).to(torch.bfloat16).cuda()
    w = torch.randn(16, 512, device="cuda")
    runs = {}
    saved = (layers.RES_BN_FUSE, layers.DS_DGRAD_DEFER)
    try:
        # (fold, defer): the shortcut's strided dgrad deferred behind the other branch's
        # (GradLink.deferred_dgrad) or run first with the zero fill — the unfolded, undeferred
        # block is the reference for both
        for fold, defer in ((False, False), (True, True), (True, False)):
            layers.RES_BN_FUSE, layers.DS_DGRAD_DEFER = fold, defer
            blk = copy.deepcopy(base).cuda()
            FusedSGD(blk.parameters(), lr=0.1).zero_grad()
            xg = x.clone().requires_grad_(True)
            h = blk.forward_fused(xg)
            (global_avg_pool(h).float() * w).sum().backward()
            torch.cuda.synchronize()
            runs[(fold, defer)] = (h.float(), xg.grad.float(),
                                   [p.grad.clone() for p in blk.parameters()],
                                   [b.clone() for b in blk.buffers() if b.dtype.is_floating_point])
    finally:
        layers.RES_BN_FUSE, layers.DS_DGRAD_DEFER = saved

    def cos(a, b):
        a, b = a.reshape(-1).double(), b.reshape(-1).double()
        return float(torch.dot(a, b) / (a.norm() * b.norm() + 1e-30))
    h0, dx0, g0, b0 = runs[(False, False)]
    names = [n for n, _ in base.named_parameters()]
    for key in ((True, True), (True, False)):
        h1, dx1, g1, b1 = runs[key]
        assert float((h1 - h0).abs().max()) <= 0.0625 * float(h0.abs().max())  # bf16 ulps
        assert cos(h1, h0) > 0.9999
        assert cos(dx1, dx0) > 0.999, key
        worst = min((cos(a, b), n) for a, b, n in zip(g1, g0, names))
        assert worst[0] > 0.998, (key, worst)
        for a, b in zip(b1, b0):
            assert torch.allclose(a, b, rtol=1e-3, atol=1e-4)


@pytest.mark.parametrize("cuts", [[8, 14], [4, 8, 14]])
def test_resnet_segmented_ddp_step_matches_single_graph(native_ext, cuts):
    """Pipelined DDP step on ResNet-50 (backward cut at block boundaries: bucket all-reduce +
    optimizer update of each segment on the comm stream, a 32-CU stand-in collective at world
    1) applies the same update as the single-graph step from the same state, eager and
    replayed, and advances the data cursor exactly once."""
    from ddp_amd.models.resnet import resnet50
    from ddp_amd.engine import CrossEntropyLoss, TrainStep, SegmentedDDPStep
    from ddp_amd.optim import FusedSGD
    from ddp_amd.data import SyntheticImageNet, DeviceLoader
    from ddp_amd.parallel import DistributedDataParallel, RcclCommunicator
    torch.manual_seed(11)
    m = DistributedDataParallel(resnet50().cuda(), RcclCommunicator(0, 1, 0), bucket_cap_mb=256.0,
                                first_bucket_cap_mb=256.0)
    opt = FusedSGD(m.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
    ld = DeviceLoader(SyntheticImageNet(True, n=64), 16, "cuda", cpad=8)
    crit = CrossEntropyLoss()
    ts = TrainStep(m, opt, crit, ld)
    ss = SegmentedDDPStep(m, opt, crit, ld, split=cuts, emulate_gbps=171.0)
    ss.WAIT_TIMEOUT_S = 20.0
    assert len(ss.buckets) == len(cuts) + 1
    # buckets tile the arena back to front
    assert ss.buckets[0][1][1] == m.arena.total and ss.buckets[-1][1][0] == 0
    for a, b in zip(ss.buckets, ss.buckets[1:]):
        assert a[1][0] == b[1][1] and a[0][0] == b[0][1]
    ts.warmup(2)
    torch.cuda.synchronize()
    snap = (m.arena.data.clone(), opt.momentum_buffer.clone(), ld.cursor.clone(),
            [b.clone() for b in m.module.buffers()])

    def run(fn):
        m.arena.data.copy_(snap[0]); opt.momentum_buffer.copy_(snap[1]); ld.cursor.copy_(snap[2])
        for b, s in zip(m.module.buffers(), snap[3]):
            b.copy_(s)
        m.arena.grad.zero_()
        for sp in m.module.fused_plan():
            sp._packed_version = None
            sp.maybe_pack()
        torch.cuda.synchronize()
        fn()
        torch.cuda.synchronize()
        assert int(ld.cursor.item()) == int(snap[2].item()) + 1
        return m.arena.data - snap[0]

    def cos(a, b):
        return float(torch.dot(a, b) / (a.norm() * b.norm()))

    # The single-graph step is itself not bit-reproducible (fp32 atomics in the BN statistics
    # flip bf16 roundings that a 50-layer network at init amplifies: two identical runs agree
    # only to cos ~0.86-0.90 here). A correct pipelined step is another sample of the same
    # distribution: compare it with the closest of three references against the spread of the
    # references among themselves.
    refs = [run(ts._body) for _ in range(3)]
    base = min(cos(refs[i], refs[j]) for i in range(3) for j in range(i + 1, 3))
    ref = refs[0]
    seg = run(ss._body)
    ss.warmup(1)
    ss.capture()
    graph = run(ss.step)
    assert float(ref.norm()) > 0
    for d in (seg, graph):
        best = max(cos(r, d) for r in refs)
        assert best > min(0.99, base - 0.03), (best, base)
        assert abs(float(d.norm()) / float(ref.norm()) - 1) < 0.03
    ss.check_error()
    m.close()


def test_resnet50_trajectory_tracks_fp32_reference(native_ext):
    """10 SGD steps (lr 0.01, momentum 0.9, wd 1e-4, batch 32, 224x224) of the fused bf16
    ResNet-50 vs the same module run through plain PyTorch (fp32 ATen/MIOpen) on the GPU, same
    weights and batches: per-step losses within a few percent, parameters aligned
    (tools/resnet_traj_check.py; at the bench's lr 0.1 both runs are chaotic on this data)."""
    import sys
    import os
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    from resnet_traj_check import ref_forward
    from ddp_amd.models.resnet import resnet50
    from ddp_amd.optim import FusedSGD
    from ddp_amd.engine import CrossEntropyLoss
    torch.manual_seed(0)
    base = resnet50()
    ref = copy.deepcopy(base).cuda()
    fus = copy.deepcopy(base).cuda()
    o_ref = torch.optim.SGD(ref.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
    o_fus = FusedSGD(fus.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
    crit = CrossEntropyLoss()
    g = torch.Generator(device="cuda").manual_seed(5)
    means = 0.25 * torch.randn(1000, 3, 1, 1, device="cuda", generator=g)
    rel = []
    for _ in range(10):
        y = torch.randint(0, 1000, (32,), device="cuda", generator=g)
        x = (torch.randn(32, 3, 224, 224, device="cuda", generator=g) + means[y]).to(torch.bfloat16).float()
        o_ref.zero_grad()
        lr_ = torch.nn.functional.cross_entropy(ref_forward(ref, x), y)
        lr_.backward()
        o_ref.step()
        o_fus.zero_grad()
        lf = crit(fus(x), y)
        lf.backward()
        o_fus.step()
        rel.append(abs(float(lf) - float(lr_)) / float(lr_))
    pr = torch.cat([p.detach().reshape(-1) for p in ref.parameters()]).double()
    pf = torch.cat([p.detach().float().reshape(-1) for p in fus.parameters()]).double()
    cos_p = float(torch.dot(pr, pf) / (pr.norm() * pf.norm()))
    print("rel loss diffs", [round(r, 4) for r in rel], "param cosine", cos_p)
    # (on the box: batch 64, 20 steps: per-step within 3 %, parameter cosine 0.9964; batch 16:
    # the first 7 steps within 1.1 %, single later steps up to 6 % — small-batch BN noise;
    # batch 32 on a fresh box: one early step at 3.1 %, mean 0.9 %, parameter cosine 0.9975.
    # Run-to-run spread of the worst early step (fp32 atomics order the BN sums differently
    # every run): 0.015-0.053 over 8 runs, mean 0.4-1.2 %, profiles/r5al_res_bn_fold.md)
    assert max(rel[:6]) < 0.08 and sum(rel) / len(rel) < 0.03 and max(rel) < 0.1, rel
    assert cos_p > 0.99, cos_p


@pytest.mark.parametrize("batch", [64])
def test_resnet50_graph_replay_matches_eager_steps(native_ext, batch):
    """Replayed ResNet-50 training steps (hipGraph) at lr 0 give the eager steps' loss for the
    same batch and leave every parameter finite. Regression: the strided 1x1 dgrad cleared its
    untouched phases with hipMemsetAsync; captured, that node did not order before the readers,
    and replays sporadically fed NaN gradients into stem..layer2 (tools/probes/resnet_graph_probe.py)."""
    import ddp_amd
    from ddp_amd.models import build
    from ddp_amd.engine import CrossEntropyLoss
    from ddp_amd.engine.step import TrainStep
    from ddp_amd.optim import FusedSGD
    from ddp_amd.data import SyntheticImageNet, DeviceLoader
    dev = torch.device("cuda", 0)
    torch.manual_seed(ddp_amd.SEED)
    loader = DeviceLoader(SyntheticImageNet(True, n=4 * batch), batch, dev, 1, 0, train=True, cpad=8)
    model = build("resnet50").to(dev)
    opt = FusedSGD(model.parameters(), lr=0.0, momentum=0.9, weight_decay=1e-4)
    step = TrainStep(model, opt, CrossEntropyLoss(), loader, use_graph=True)
    eager = []
    for _ in range(4):  # one pass over the 4 batches of the dataset
        step.warmup(1)
        eager.append(step.pop_loss())
    step.capture()
    step.pop_loss()
    for i in range(8):  # two more passes, replayed
        step.step()
        v = step.pop_loss()
        assert v == v and abs(v - eager[i % 4]) < 2e-2 * abs(eager[i % 4]), (i, v, eager)
    assert bool(torch.isfinite(opt.arena.data).all())
    assert bool(torch.isfinite(opt.momentum_buffer).all())
