"""Flat parameter arena: [K][R][S][C] conv-weight storage keeps the reference state_dict contract."""
import torch


def test_krsc_arena_views_and_state_dict():
    from ddp_amd.models import VGG11
    from ddp_amd.optim.arena import ParamArena
    torch.manual_seed(0)
    m = VGG11()
    ref = {k: v.clone() for k, v in m.state_dict().items()}
    a = ParamArena(list(m.parameters()), device="cpu", krsc=True)
    w = m.layers[4].weight  # 128 x 64 x 3 x 3
    i = a.index(w)
    assert a.krsc[i] and not a.krsc[a.index(m.fc1.weight)]
    assert w.shape == (128, 64, 3, 3) and w.is_contiguous(memory_format=torch.channels_last)
    o, n = a.offsets[i], a.numels[i]
    assert torch.equal(a.data[o:o + n], ref["layers.4.weight"].permute(0, 2, 3, 1).reshape(-1))
    for k, v in m.state_dict().items():
        assert torch.equal(v, ref[k]), k
    # grads are views with the same layout; writes through them land in the flat arena
    w.grad.fill_(1.0)
    assert float(a.grad[o:o + n].sum()) == n
    # load_state_dict writes through the permuted views
    m2 = VGG11()
    m.load_state_dict(m2.state_dict())
    assert torch.equal(a.data[o:o + n], m2.layers[4].weight.detach().permute(0, 2, 3, 1).reshape(-1))
    # relink after .data was replaced by a contiguous tensor
    w.data = torch.full((128, 64, 3, 3), 2.0)
    a.relink()
    assert w.data_ptr() == a.data[o:o + n].data_ptr() and float(a.data[o:o + n].mean()) == 2.0
    # forward still matches the reference-layout model
    x = torch.randn(2, 3, 32, 32)
    m2.load_state_dict(m.state_dict())
    assert torch.allclose(m(x), m2(x), atol=1e-5)
