"""Synthetic datasets, sharded sampling and (on-device) augmentation."""
from .synthetic import SyntheticCIFAR10, SyntheticImageNet, SyntheticImageDataset  # noqa: F401
from .loader import (CPULoader, DeviceLoader, make_loader, shard_indices, augment_cpu,  # noqa: F401
                     CIFAR_MEAN, CIFAR_STD)
