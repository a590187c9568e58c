"""Deterministic synthetic datasets (CIFAR-10-shaped and ImageNet-shaped).

Reference parity: torchvision ``datasets.CIFAR10(root, train, download=True)`` (part1/main.py:34-43).
Neither torchvision nor a network exists on the GPU boxes, so images are
generated from a seed with a counter-based hash. Every image = 5/8 class template + 3/8 per-image
noise, so the classification task is learnable (loss goes down) while remaining fully
reproducible. The exact same integer formula is implemented on the GPU in
csrc/kernels/data.hip (``synth_pixel`` / ``synth_label``); tests check they agree bit for bit.
"""
import numpy as np
import torch

M32 = np.uint32(0xFFFFFFFF)


def hash_u32(x):
    x = np.asarray(x, dtype=np.uint32).copy()
    x ^= x >> np.uint32(16)
    x *= np.uint32(0x7feb352d)
    x ^= x >> np.uint32(15)
    x *= np.uint32(0x846ca68b)
    x ^= x >> np.uint32(16)
    return x


def hash3(a, b, c):
    a = np.asarray(a, dtype=np.uint32)
    b = np.asarray(b, dtype=np.uint32)
    c = np.asarray(c, dtype=np.uint32)
    with np.errstate(over="ignore"):
        return hash_u32(a ^ hash_u32(b ^ hash_u32(c + np.uint32(0x9e3779b9))))


def synth_labels(seed, idx, classes):
    return (hash3(np.uint32(seed), np.asarray(idx, dtype=np.uint32), np.uint32(0xabcdef)) %
            np.uint32(classes)).astype(np.int64)


def synth_images(seed, idx, labels, pix_per_img):
    """uint8 [len(idx), pix_per_img] (HWC order within an image)."""
    idx = np.asarray(idx, dtype=np.uint32)[:, None]
    lab = np.asarray(labels, dtype=np.uint32)[:, None]
    p = np.arange(pix_per_img, dtype=np.uint32)[None, :]
    t = hash3(np.uint32(seed), np.uint32(0x1000) + lab, p) & np.uint32(255)
    u = hash3(np.uint32(seed) ^ np.uint32(0x5bd1e995), idx, p) & np.uint32(255)
    return ((t * np.uint32(5) + u * np.uint32(3)) >> np.uint32(3)).astype(np.uint8)


class SyntheticImageDataset:
    """Synthetic labelled images, materialised lazily on CPU (numpy) or on a GPU (HIP kernel)."""

    def __init__(self, n, height=32, width=32, classes=10, seed=89395, name="synthetic"):
        self.n, self.height, self.width, self.classes, self.seed = n, height, width, classes, seed
        self.name = name
        self._cpu = None
        self._dev = {}

    def __len__(self):
        return self.n

    @property
    def pix_per_img(self):
        return self.height * self.width * 3

    def cpu_arrays(self, chunk=4096):
        """(images uint8 [n, H, W, 3], labels int64 [n]) generated with numpy."""
        if self._cpu is None:
            labels = synth_labels(self.seed, np.arange(self.n), self.classes)
            imgs = np.empty((self.n, self.pix_per_img), dtype=np.uint8)
            for s in range(0, self.n, chunk):
                e = min(self.n, s + chunk)
                imgs[s:e] = synth_images(self.seed, np.arange(s, e), labels[s:e], self.pix_per_img)
            self._cpu = (imgs.reshape(self.n, self.height, self.width, 3), labels)
        return self._cpu

    def device_arrays(self, device):
        """(images uint8 [n, H, W, 3], labels int32 [n]) generated on the GPU."""
        key = str(device)
        if key not in self._dev:
            from ..ops.common import native, stream_handle
            imgs = torch.empty(self.n, self.height, self.width, 3, dtype=torch.uint8, device=device)
            labels = torch.empty(self.n, dtype=torch.int32, device=device)
            native().synth_generate(imgs.data_ptr(), labels.data_ptr(), self.n, self.pix_per_img,
                                    self.seed & 0xFFFFFFFF, self.classes, stream_handle())
            self._dev[key] = (imgs, labels)
        return self._dev[key]


def SyntheticCIFAR10(train=True, seed=89395, n=None):
    """CIFAR-10-shaped: 50 000 train / 10 000 test images of 3x32x32, 10 classes."""
    n = n if n is not None else (50000 if train else 10000)
    return SyntheticImageDataset(n, 32, 32, 10, seed if train else seed + 1,
                                 name="cifar10-train" if train else "cifar10-test")


def SyntheticImageNet(train=True, seed=89395, n=None, size=224):
    """ImageNet-shaped: 3x224x224, 1000 classes (driver's ResNet-50 config)."""
    n = n if n is not None else (2048 if train else 512)
    return SyntheticImageDataset(n, size, size, 1000, seed if train else seed + 1,
                                 name="imagenet-train" if train else "imagenet-test")
