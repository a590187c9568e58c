"""ResNet-50 (driver config) on the gfx950 path vs the CPU fp32 ATen oracle."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_resnet50_train_step_matches_cpu(native_ext):
    from ddp_amd.models.resnet import resnet50
    from ddp_amd.engine import CrossEntropyLoss
    from ddp_amd.optim import FusedSGD
    torch.manual_seed(0)
    cpu = resnet50(num_classes=16)
    gpu = copy.deepcopy(cpu).cuda()
    opt = FusedSGD(gpu.parameters(), lr=0.1)
    x = torch.randn(8, 3, 64, 64).to(torch.bfloat16).float()
    y = torch.randint(0, 16, (8,))
    crit = CrossEntropyLoss()
    lc = crit(cpu(x), y)
    lc.backward()
    opt.zero_grad()
    out = gpu(x.cuda())
    assert out.shape == (8, 16)
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
    assert min(cos.values()) > 0.8, min(cos.items(), key=lambda kv: kv[1])
    assert cos["fc.weight"] > 0.99
    # eval mode uses running statistics
    gpu.eval()
    cpu.eval()
    with torch.no_grad():
        oe_g, oe_c = gpu(x.cuda()).float().cpu(), cpu(x)
    assert float((oe_g - oe_c).norm() / oe_c.norm()) < 0.1
