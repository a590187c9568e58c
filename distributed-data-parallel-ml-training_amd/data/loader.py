"""Sharded sampling, augmentation and batch loaders.

Reference parity (part1/main.py:19-50, part2/part2a/main.py:61-94, part3/main.py:62-95):
* train transform: RandomCrop(32, padding=4) -> RandomHorizontalFlip() -> ToTensor() ->
  Normalize(mean=[125.3,123.0,113.9]/255, std=[63.0,62.1,66.7]/255); test: ToTensor + Normalize;
* ``DistributedSampler(num_replicas=ws, rank=rank, shuffle=False, drop_last=False)`` shards the
  training set; the test loader is NOT sharded (every rank evaluates the whole test set).
  We use torch's own DistributedSampler for the index arithmetic (padding / strided shards).

Two loaders with identical semantics:
* ``DeviceLoader`` (GPU): the dataset lives in HBM as uint8; one fused HIP kernel per batch
  gathers the rank's samples, applies crop/flip/normalise and writes NHWC bf16 (3 real + 5 zero
  channels) plus int64 labels — no worker processes, no host->device copies. A device-side
  cursor lets the augment kernel live inside a replayed hipGraph (``static_batch``/``fill``).
* ``CPULoader`` (CPU): numpy implementation of the same per-sample crop/flip decisions (same
  hash), producing NCHW fp32 like ToTensor+Normalize — the oracle for the GPU kernel.
Per-sample randomness is hash(seed, epoch, sample index): independent of rank and world size.
"""
import math

import numpy as np
import torch
from torch.utils.data.distributed import DistributedSampler

from .synthetic import hash3

CIFAR_MEAN = [x / 255.0 for x in [125.3, 123.0, 113.9]]
CIFAR_STD = [x / 255.0 for x in [63.0, 62.1, 66.7]]
AUG_SEED_XOR = 0x68e31da4


class _Len:
    def __init__(self, n):
        self.n = n

    def __len__(self):
        return self.n


def shard_indices(n, num_replicas=1, rank=0, shuffle=False, drop_last=False, epoch=0, seed=0):
    """Indices of this rank's shard, exactly as torch's DistributedSampler produces them."""
    s = DistributedSampler(_Len(n), num_replicas=num_replicas, rank=rank, shuffle=shuffle,
                           drop_last=drop_last, seed=seed)
    s.set_epoch(epoch)
    return list(iter(s))


def crop_flip_params(seed, epoch, idx, pad=4, flip=True):
    h = hash3(np.uint32(seed) ^ np.uint32(AUG_SEED_XOR), np.uint32(epoch), np.asarray(idx, np.uint32))
    span = 2 * pad + 1
    cy = (h % np.uint32(span)).astype(np.int64)
    cx = ((h // np.uint32(span)) % np.uint32(span)).astype(np.int64)
    fl = ((h >> np.uint32(20)) & np.uint32(1)).astype(np.int64) if flip else np.zeros_like(cy)
    return cy, cx, fl


def augment_cpu(images, idx, seed, epoch, train=True, pad=4, mean=CIFAR_MEAN, std=CIFAR_STD):
    """NCHW fp32 batch for sample indices ``idx`` (numpy twin of the HIP augment kernel)."""
    idx = np.asarray(idx)
    x = images[idx].astype(np.float32)  # [B, H, W, 3]
    B, H, W, _ = x.shape
    if train:
        cy, cx, fl = crop_flip_params(seed, epoch, idx, pad, True)
        padded = np.zeros((B, H + 2 * pad, W + 2 * pad, 3), dtype=np.float32)
        padded[:, pad:pad + H, pad:pad + W] = x
        out = np.empty_like(x)
        for b in range(B):
            crop = padded[b, cy[b]:cy[b] + H, cx[b]:cx[b] + W]
            out[b] = crop[:, ::-1] if fl[b] else crop
        x = out
    x = x / 255.0
    x = (x - np.asarray(mean, np.float32)) / np.asarray(std, np.float32)
    return torch.from_numpy(np.ascontiguousarray(x.transpose(0, 3, 1, 2)))


class CPULoader:
    def __init__(self, dataset, batch_size, num_replicas=1, rank=0, train=True, shard=True,
                 epoch=0, max_batches=None):
        self.ds, self.batch_size, self.train = dataset, batch_size, train
        self.num_replicas = num_replicas if shard else 1
        self.rank = rank if shard else 0
        self.epoch = epoch
        self.max_batches = max_batches

    def set_epoch(self, e):
        self.epoch = e

    def indices(self):
        return shard_indices(len(self.ds), self.num_replicas, self.rank, epoch=self.epoch)

    def __len__(self):
        n = math.ceil(len(self.indices()) / self.batch_size)
        return min(n, self.max_batches) if self.max_batches else n

    @property
    def dataset(self):
        return self.ds

    def __iter__(self):
        imgs, labels = self.ds.cpu_arrays()
        idx = self.indices()
        for bi, s in enumerate(range(0, len(idx), self.batch_size)):
            if self.max_batches and bi >= self.max_batches:
                break
            b = idx[s:s + self.batch_size]
            yield augment_cpu(imgs, b, self.ds.seed, self.epoch, self.train), \
                torch.from_numpy(labels[b].astype(np.int64))


class DeviceLoader:
    def __init__(self, dataset, batch_size, device, num_replicas=1, rank=0, train=True,
                 shard=True, epoch=0, max_batches=None, cpad=8):
        self.ds, self.batch_size, self.train = dataset, batch_size, train
        self.device = torch.device(device)
        self.num_replicas = num_replicas if shard else 1
        self.rank = rank if shard else 0
        self.max_batches = max_batches
        self.cpad = cpad
        self.images, self.labels = dataset.device_arrays(self.device)
        self.cursor = torch.zeros(1, dtype=torch.int32, device=self.device)
        self._static = None
        self.set_epoch(epoch)

    @property
    def dataset(self):
        return self.ds

    def set_epoch(self, e):
        self.epoch = e
        idx = torch.tensor(shard_indices(len(self.ds), self.num_replicas, self.rank, epoch=e),
                           dtype=torch.int32)
        if getattr(self, "idx", None) is not None and self.idx.numel() == idx.numel():
            self.idx.copy_(idx)  # in place: a captured step keeps pointing at live memory
        else:
            self.idx = idx.to(self.device)
        self.cursor.zero_()

    def __len__(self):
        n = math.ceil(self.idx.numel() / self.batch_size)
        return min(n, self.max_batches) if self.max_batches else n

    def _launch(self, x, y, indices_ptr, L, B, cursor_ptr):
        from ..ops.common import native, stream_handle, step_scratch
        pad, flip = (4, 1) if self.train else (0, 0)
        # the augment launch also clears the per-step BN-statistics scratch that the next
        # forward would otherwise zero with a fill kernel of its own (StepScratch.zero)
        sc = step_scratch(self.device)
        zp, zn = sc.claim_zero()
        native().augment(self.images.data_ptr(), self.labels.data_ptr(), indices_ptr, cursor_ptr,
                         L, B, self.ds.height, self.ds.width, self.cpad, pad, flip,
                         self.ds.seed & 0xFFFFFFFF, self.epoch, CIFAR_MEAN, CIFAR_STD,
                         x.data_ptr(), y.data_ptr(), stream_handle(), zero=zp, zero_n=zn)

    def batch(self, start, B):
        """Materialise samples [start, start+B) of this rank's shard (new tensors)."""
        x = torch.empty(B, self.ds.height, self.ds.width, self.cpad, dtype=torch.bfloat16,
                        device=self.device)
        y = torch.empty(B, dtype=torch.int64, device=self.device)
        self._launch(x, y, self.idx.data_ptr() + 4 * start, B, B, 0)
        return x, y

    def __iter__(self):
        L = self.idx.numel()
        for bi, s in enumerate(range(0, L, self.batch_size)):
            if self.max_batches and bi >= self.max_batches:
                break
            yield self.batch(s, min(self.batch_size, L - s))

    # ---- graph-capturable form: fixed-shape static buffers + device cursor
    def static_batch(self):
        if self._static is None:
            B = self.batch_size
            x = torch.empty(B, self.ds.height, self.ds.width, self.cpad, dtype=torch.bfloat16,
                            device=self.device)
            y = torch.empty(B, dtype=torch.int64, device=self.device)
            self._static = (x, y)
        return self._static

    def fill(self, advance=True):
        """Write the next batch (cursor-addressed, wraps around the shard) into the static
        buffers and advance the device cursor. Safe to capture into a hipGraph.
        ``advance=False`` leaves the increment to the caller (engine/step.py folds it into the
        optimizer launch: see ``cursor_advance``)."""
        from ..ops.common import native, stream_handle
        x, y = self.static_batch()
        self._launch(x, y, self.idx.data_ptr(), self.idx.numel(), self.batch_size,
                     self.cursor.data_ptr())
        if advance:
            native().counter_add(self.cursor.data_ptr(), 1, stream_handle())
        return x, y

    def cursor_advance(self):
        """(device pointer, delta) of the pending cursor increment after ``fill(advance=False)``."""
        return (self.cursor.data_ptr(), 1)


def make_loader(dataset, batch_size, device, num_replicas=1, rank=0, train=True, shard=True,
                max_batches=None):
    if torch.device(device).type == "cuda":
        return DeviceLoader(dataset, batch_size, device, num_replicas, rank, train, shard,
                            max_batches=max_batches)
    return CPULoader(dataset, batch_size, num_replicas, rank, train, shard, max_batches=max_batches)
