"""Synthetic data, sharded sampling and the CPU augmentation oracle."""
import numpy as np
import torch

from ddp_amd.data import SyntheticCIFAR10, CPULoader, shard_indices, augment_cpu
from ddp_amd.data.synthetic import hash_u32


def test_hash_known_values():
    # fixed points of the formula shared with csrc/kernels/common.h (guards silent changes)
    v = hash_u32(np.array([0, 1, 2, 0xFFFFFFFF], dtype=np.uint32))
    assert v.dtype == np.uint32
    assert v[0] == 0
    assert len(set(v.tolist())) == 4


def test_dataset_deterministic_and_learnable():
    a = SyntheticCIFAR10(True, n=200).cpu_arrays()
    b = SyntheticCIFAR10(True, n=200).cpu_arrays()
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    imgs, labels = a
    assert imgs.shape == (200, 32, 32, 3) and imgs.dtype == np.uint8
    assert set(labels.tolist()) <= set(range(10)) and len(set(labels.tolist())) == 10
    # same-class images are closer to each other than to other classes (template structure)
    m = [imgs[labels == c].reshape(-1, 3072).mean(0) for c in range(10)]
    x0 = imgs[0].reshape(-1).astype(np.float32)
    d = [np.abs(x0 - mc).mean() for mc in m]
    assert int(np.argmin(d)) == labels[0]
    test = SyntheticCIFAR10(False, n=50).cpu_arrays()[0]
    assert not np.array_equal(test[:50], imgs[:50])


def test_shard_indices_reference_semantics():
    # DistributedSampler(shuffle=False, drop_last=False): pad by wrapping, strided shards
    n, w = 10, 4
    shards = [shard_indices(n, w, r) for r in range(w)]
    assert shards[0] == [0, 4, 8]
    assert shards[1] == [1, 5, 9]
    assert shards[2] == [2, 6, 0]
    assert shards[3] == [3, 7, 1]
    assert shard_indices(50000, 1, 0) == list(range(50000))


def test_augment_cpu_crop_flip_normalize():
    imgs, _ = SyntheticCIFAR10(True, n=16).cpu_arrays()
    x = augment_cpu(imgs, np.arange(16), 7, 0, train=False)
    mean = np.array([125.3, 123.0, 113.9]) / 255
    std = np.array([63.0, 62.1, 66.7]) / 255
    exp = (imgs[3].astype(np.float32) / 255 - mean) / std
    assert np.allclose(x[3].numpy().transpose(1, 2, 0), exp, atol=1e-5)
    xa = augment_cpu(imgs, np.arange(16), 7, 0, train=True)
    assert xa.shape == (16, 3, 32, 32)
    # every augmented image is a crop (+maybe flip) of the zero-padded original
    pad_val = (0 - mean) / std
    for b in range(16):
        img = xa[b].numpy().transpose(1, 2, 0)
        orig = (imgs[b].astype(np.float32) / 255 - mean) / std
        P = np.tile(pad_val, (40, 40, 1)).astype(np.float32)
        P[4:36, 4:36] = orig
        found = False
        for cy in range(9):
            for cx in range(9):
                c = P[cy:cy + 32, cx:cx + 32]
                if np.allclose(c, img, atol=1e-5) or np.allclose(c[:, ::-1], img, atol=1e-5):
                    found = True
                    break
            if found:
                break
        assert found, b


def test_cpu_loader_shapes_and_sharding():
    ds = SyntheticCIFAR10(True, n=100)
    ld = CPULoader(ds, 16, num_replicas=2, rank=1)
    batches = list(ld)
    assert len(batches) == len(ld) == 4  # 50 samples per rank -> 16,16,16,2
    assert batches[0][0].shape == (16, 3, 32, 32) and batches[0][0].dtype == torch.float32
    assert batches[-1][0].shape[0] == 2
    _, labels = ds.cpu_arrays()
    assert torch.equal(batches[0][1], torch.from_numpy(labels[1:32:2]))
