"""Data layer (reference data.py): MNIST-shaped data, DistributedSampler-exact sharding,
the reference's CPU DataLoader and the HBM-resident device loader."""
from .imagenet import DeviceImageLoader, DeviceImages, synthetic_imagenet
from .loader import DeviceMNIST, DeviceMNISTLoader, get_dataloader
from .mnist import MNISTDataset, load_mnist, mnist_available, read_idx, synthetic_mnist
from .sampler import ShardedSampler, epoch_indices, num_samples, steps_per_epoch

__all__ = ["DeviceImageLoader", "DeviceImages", "synthetic_imagenet", "DeviceMNIST", "DeviceMNISTLoader", "get_dataloader", "MNISTDataset", "load_mnist",
           "mnist_available", "read_idx", "synthetic_mnist", "ShardedSampler", "epoch_indices",
           "num_samples", "steps_per_epoch"]
