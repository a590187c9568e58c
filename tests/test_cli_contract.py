"""CLI / model / checkpoint contract with the reference."""
import os
import subprocess
import sys

import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# reference state_dict layout
CONV_IDX = [0, 4, 8, 11, 15, 18, 22, 25]
BN_IDX = [1, 5, 9, 12, 16, 19, 23, 26]
CONV_SHAPES = [(64, 3, 3, 3), (128, 64, 3, 3), (256, 128, 3, 3), (256, 256, 3, 3),
               (512, 256, 3, 3), (512, 512, 3, 3), (512, 512, 3, 3), (512, 512, 3, 3)]


def test_parse_arguments_defaults(monkeypatch):
    from ddp_amd.utils.cli import parse_arguments
    for k in ("RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        monkeypatch.delenv(k, raising=False)
    ip, port, rank, size = parse_arguments(["--num-nodes", "4", "--rank", "2"])
    assert (ip, port, rank, size) == ("10.10.1.1", "4000", 2, 4)
    assert isinstance(port, str)


def test_rank_default_is_lazy_and_non_fatal(monkeypatch):
    from ddp_amd.utils import cli
    monkeypatch.delenv("RANK", raising=False)
    monkeypatch.setattr(cli.os, "uname", lambda: type("U", (), {"nodename": "localhost"})())
    assert cli.get_rank() == 0  # reference would raise ValueError here
    monkeypatch.setattr(cli.os, "uname", lambda: type("U", (), {"nodename": "node3.cluster"})())
    assert cli.get_rank() == 3
    monkeypatch.setenv("RANK", "5")
    assert cli.get_rank() == 5


def test_flag_names_and_dests():
    from ddp_amd.utils.cli import build_parser
    p = build_parser()
    acts = {a.dest: a for a in p._actions}
    assert acts["master_ip"].option_strings == ["--master-ip"]
    assert acts["master_port"].option_strings == ["--master-port"]
    assert acts["size"].option_strings == ["--num-nodes"] and acts["size"].type is int
    assert acts["rank"].option_strings == ["--rank"] and acts["rank"].type is int


def test_vgg11_state_dict_layout():
    from ddp_amd.models import VGG11
    sd = VGG11().state_dict()
    exp = {}
    for i, s in zip(CONV_IDX, CONV_SHAPES):
        exp[f"layers.{i}.weight"] = s
        exp[f"layers.{i}.bias"] = (s[0],)
    for i, s in zip(BN_IDX, CONV_SHAPES):
        exp[f"layers.{i}.weight"] = (s[0],)
        exp[f"layers.{i}.bias"] = (s[0],)
    exp["fc1.weight"] = (10, 512)
    exp["fc1.bias"] = (10,)
    assert {k: tuple(v.shape) for k, v in sd.items()} == exp
    assert len(list(VGG11().parameters())) == 34
    assert sum(p.numel() for p in VGG11().parameters()) == 9231114


@pytest.mark.skipif(not os.path.exists("/root/reference/part1/model.py"), reason="no reference")
def test_state_dict_loads_into_reference_model(tmp_path):
    import importlib.util
    spec = importlib.util.spec_from_file_location("ref_model", "/root/reference/part1/model.py")
    ref = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ref)
    from ddp_amd.models import VGG11
    from ddp_amd.utils import save_checkpoint
    m = VGG11()
    path = str(tmp_path / "ck.pt")
    save_checkpoint(path, m)
    obj = torch.load(path, weights_only=True)
    r = ref.VGG11()
    r.load_state_dict(obj["model"])  # strict: identical keys and shapes
    x = torch.randn(4, 3, 32, 32)
    assert torch.allclose(r(x), m(x), atol=1e-5)


def test_checkpoint_roundtrip_with_ddp_prefix(tmp_path):
    from ddp_amd.models import VGG11
    from ddp_amd.utils import save_checkpoint, load_checkpoint
    a, b = VGG11(), VGG11()

    class Wrap(torch.nn.Module):
        def __init__(self, m):
            super().__init__()
            self.module = m
    path = str(tmp_path / "c.pt")
    save_checkpoint(path, Wrap(a))
    load_checkpoint(path, b)
    for (k, x), (_, y) in zip(a.state_dict().items(), b.state_dict().items()):
        assert torch.equal(x, y), k


def test_part_mains_exist_and_export_vgg11():
    for p in ["part1", "part2/part2a", "part2/part2b", "part3"]:
        assert os.path.exists(os.path.join(REPO, p, "main.py"))
        assert os.path.exists(os.path.join(REPO, p, "model.py"))
    sys.path.insert(0, os.path.join(REPO, "part3"))
    try:
        import importlib
        mm = importlib.import_module("model")
        assert hasattr(mm, "VGG11") and hasattr(mm, "_cfg") and hasattr(mm, "_make_layers")
    finally:
        sys.path.pop(0)


def test_part1_cpu_output_format():
    r = subprocess.run([sys.executable, os.path.join(REPO, "part1", "main.py"), "--device", "cpu",
                        "--train-size", "640", "--test-size", "64", "--max-batches", "41",
                        "--global-batch", "8", "--threads", "2"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr
    out = r.stdout.splitlines()
    assert any(l.startswith("[1,    20] loss: ") for l in out)
    assert any(l.startswith("[1,    40] loss: ") for l in out)
    assert any(l.startswith("Total time for 1-39 iteration in ns: ") for l in out)
    assert any(l.startswith("Average time for 1-39 iteration in ns: ") for l in out)
    assert any(l.startswith("Test set: Average loss: ") and "Accuracy: " in l and "/64 (" in l for l in out)


def test_resnet50_layout_cpu():
    from ddp_amd.models.resnet import resnet50
    m = resnet50()
    params = list(m.parameters())
    assert len(params) == 161
    assert sum(p.numel() for p in params) == 25557032
    sd = m.state_dict()
    for k in ["conv1.weight", "bn1.running_mean", "bn1.num_batches_tracked",
              "layer1.0.downsample.0.weight", "layer4.2.bn3.bias", "fc.weight", "fc.bias"]:
        assert k in sd, k
    with torch.no_grad():
        out = m(torch.randn(1, 3, 64, 64))
    assert out.shape == (1, 1000)
