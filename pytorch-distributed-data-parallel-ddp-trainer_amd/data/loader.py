"""Data loaders: the reference's CPU ``DataLoader`` and the HBM-resident device loader.

Reference (data.py:6-27): ``get_dataloader(batch_size, world_size, rank)`` builds
``DataLoader(MNIST, batch_size, sampler=DistributedSampler(..., shuffle=True),
num_workers=2, pin_memory=True)`` and returns ``(dataloader, sampler)``.  Every batch then
costs worker-process decode, collate and a host-to-device copy.

MI355X design: the whole uint8 training set (47 MB) lives in HBM.
Once per epoch the rank's sampler indices are uploaded as one tensor; a batch is then a
device-side gather.  The fused engine goes one step further and never materialises the
batch at all: its first convolution reads ``images_u8`` through the index list and
applies ``/255`` in registers.
"""
from __future__ import annotations

import torch

from .mnist import MNISTDataset, load_mnist
from .sampler import ShardedSampler, steps_per_epoch


class DeviceMNIST:
    """uint8 images + labels resident on one device (int32 labels for the HIP kernels)."""

    def __init__(self, images_u8: torch.Tensor, labels: torch.Tensor, device,
                 source: str = "synthetic"):
        if images_u8.dtype != torch.uint8 or images_u8.dim() != 3:
            raise ValueError(f"expected uint8 [N,H,W] images, got {images_u8.dtype} {tuple(images_u8.shape)}")
        if labels.shape[0] != images_u8.shape[0]:
            raise ValueError("images and labels differ in length")
        if labels.numel() and (int(labels.min()) < 0 or int(labels.max()) > 9):
            raise ValueError("labels must lie in [0, 9]")
        self.device = torch.device(device)
        self.source = source
        self.images_u8 = images_u8.contiguous().to(self.device)
        self.labels_i32 = labels.to(torch.int32).to(self.device)
        self.labels_i64 = labels.to(torch.int64).to(self.device)

    def __len__(self) -> int:
        return self.images_u8.shape[0]

    def gather(self, idx: torch.Tensor):
        """``(float32 [B,1,28,28] = u8/255, int64 [B])`` for device indices ``idx``."""
        x = self.images_u8.index_select(0, idx).unsqueeze(1).float().div_(255.0)
        return x, self.labels_i64.index_select(0, idx)


class DeviceMNISTLoader:
    """Iterates the rank's ``DistributedSampler``-exact batches out of HBM.

    Same length and batch contents as the reference's DataLoader (ragged last batch,
    drop_last=False); one index upload per epoch instead of one H2D copy per batch."""

    def __init__(self, data: DeviceMNIST, batch_size: int, world_size: int, rank: int,
                 shuffle: bool = True, seed: int = 0):
        self.data, self.batch_size = data, int(batch_size)
        self.sampler = ShardedSampler(len(data), world_size, rank, shuffle=shuffle, seed=seed)

    def __len__(self) -> int:
        return steps_per_epoch(len(self.data), self.sampler.num_replicas, self.batch_size)

    def __iter__(self):
        idx = self.sampler.indices().to(self.data.device, non_blocking=False)
        for s in range(0, idx.numel(), self.batch_size):
            yield self.data.gather(idx[s:s + self.batch_size])


def get_dataloader(batch_size: int, world_size: int, rank: int, root: str = "./data",
                   source: str = "auto", num_workers: int = 2, pin_memory: bool | None = None):
    """The reference's ``get_dataloader`` (data.py:6-27) → ``(DataLoader, sampler)``.

    Used by the CPU/gloo configuration; ``pin_memory`` defaults to "only when a GPU
    exists" (the reference's unconditional True warns on CPU hosts)."""
    imgs, labels, _ = load_mnist(root, source)
    dataset = MNISTDataset(imgs, labels)
    sampler = ShardedSampler(len(dataset), world_size, rank, shuffle=True)
    if pin_memory is None:
        pin_memory = torch.cuda.is_available()
    loader = torch.utils.data.DataLoader(dataset, batch_size=batch_size, sampler=sampler,
                                         num_workers=num_workers, pin_memory=pin_memory,
                                         persistent_workers=num_workers > 0)
    return loader, sampler
