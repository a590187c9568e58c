"""Whole-model checks on the GPU: VGG-11 fused gfx950 path vs the CPU fp32 oracle, and the
hipGraph-captured training step vs eager steps."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def rel(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-12))


def test_vgg11_forward_backward_matches_cpu_oracle(native_ext):
    from ddp_amd.models import VGG11
    from ddp_amd.engine import CrossEntropyLoss
    from ddp_amd.optim import FusedSGD
    torch.manual_seed(1)
    cpu = VGG11()
    gpu = copy.deepcopy(cpu).cuda()
    opt = FusedSGD(gpu.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    x = torch.randn(32, 3, 32, 32).to(torch.bfloat16).float()
    y = torch.randint(0, 10, (32,))
    crit = CrossEntropyLoss()
    lc = crit(cpu(x), y)
    lc.backward()
    opt.zero_grad()
    lg = crit(gpu(x.cuda()), y.cuda())
    lg.backward()
    torch.cuda.synchronize()
    assert abs(float(lg) - float(lc)) < 0.05 * max(1.0, abs(float(lc)))
    for (n, pc), pg in zip(cpu.named_parameters(), gpu.parameters()):
        e = rel(pg.grad.cpu(), pc.grad)
        # conv biases have an analytically-zero gradient (BN follows): compare absolutely
        if n.endswith("bias") and n.startswith("layers.") and int(n.split(".")[1]) % 4 in (0, 1) \
                and pc.grad.norm() < 1e-4:
            assert float(pg.grad.abs().max()) < 1e-3, n
            continue
        assert e < 0.1, f"{n}: rel err {e}"


def test_graph_step_equals_eager(native_ext):
    from ddp_amd.models import VGG11
    from ddp_amd.engine import CrossEntropyLoss, TrainStep
    from ddp_amd.optim import FusedSGD
    from ddp_amd.data import SyntheticCIFAR10, DeviceLoader
    ds = SyntheticCIFAR10(True, n=512)

    def make(use_graph):
        torch.manual_seed(5)
        m = VGG11().cuda()
        opt = FusedSGD(m.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4)
        ld = DeviceLoader(ds, 64, "cuda")
        return m, opt, TrainStep(m, opt, CrossEntropyLoss(), ld, use_graph=use_graph)

    m1, o1, s1 = make(False)
    m2, o2, s2 = make(True)
    s1.warmup(2)
    s2.warmup(2)
    s2.capture()
    for _ in range(3):
        s1.step()
        s2.step()
    torch.cuda.synchronize()
    # atomics make the last bits run-to-run dependent; require close agreement
    for p1, p2 in zip(m1.parameters(), m2.parameters()):
        assert rel(p2, p1) < 1e-3
    l1, l2 = s1.pop_loss(), s2.pop_loss()
    assert abs(l1 - l2) < 1e-2 * max(1, abs(l1))


def test_training_reduces_loss(native_ext):
    from ddp_amd.models import VGG11
    from ddp_amd.engine import CrossEntropyLoss, TrainStep
    from ddp_amd.optim import FusedSGD
    from ddp_amd.data import SyntheticCIFAR10, DeviceLoader
    torch.manual_seed(3)
    m = VGG11().cuda()
    opt = FusedSGD(m.parameters(), lr=0.02, momentum=0.9, weight_decay=1e-4)
    ld = DeviceLoader(SyntheticCIFAR10(True, n=2048), 128, "cuda")
    st = TrainStep(m, opt, CrossEntropyLoss(), ld)
    st.warmup(2)
    st.capture()
    first = None
    for i in range(6):
        for _ in range(10):
            st.step()
        v = st.pop_loss() / 10
        first = v if first is None else first
    assert v < first, (first, v)
