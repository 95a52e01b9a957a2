"""Synthetic ImageNet-shaped data for ResNet-18 (BASELINE.json config 5).

There is no network for ImageNet here, so the dataset is generated: ``n`` uint8 RGB
images of ``size x size`` (stored NHWC, 150 KB each at 224) with labels in
``[0, num_classes)``.  Each class has its own mean colour and the images carry seeded
per-pixel noise, so a network can fit them and the loss curve means something.

Like the MNIST loader, the set lives in HBM; a batch is a device-side gather that the
``image_gather_nhwc4`` HIP kernel turns straight into the stem's input format: NHWC bf16
with the 3 channels zero-padded to 4, scaled by 1/255 (ToTensor semantics, no
normalisation - like the reference's MNIST pipeline).  On the CPU the same data comes
out as NCHW float for the PyTorch oracle path.
"""
from __future__ import annotations

import torch

from .sampler import ShardedSampler, steps_per_epoch


def synthetic_imagenet(n: int = 2048, size: int = 224, num_classes: int = 1000, seed: int = 0):
    """``(uint8 [n, size, size, 3], int64 [n])`` - class-coloured noisy images."""
    g = torch.Generator().manual_seed(seed)
    labels = torch.randint(0, num_classes, (n,), generator=g)
    colours = torch.randint(32, 224, (num_classes, 3), generator=g, dtype=torch.int16)
    imgs = torch.empty(n, size, size, 3, dtype=torch.uint8)
    for s in range(0, n, 64):  # bounded temporaries
        e = min(n, s + 64)
        noise = torch.randint(-32, 33, (e - s, size, size, 3), generator=g, dtype=torch.int16)
        imgs[s:e] = (colours[labels[s:e]].view(-1, 1, 1, 3) + noise).clamp_(0, 255).to(torch.uint8)
    return imgs, labels


class DeviceImages:
    """uint8 NHWC images + int64 labels resident on one device."""

    def __init__(self, images_u8: torch.Tensor, labels: torch.Tensor, device):
        if images_u8.dtype != torch.uint8 or images_u8.dim() != 4 or images_u8.shape[3] != 3:
            raise ValueError(f"expected uint8 [N,H,W,3] images, got {images_u8.dtype} {tuple(images_u8.shape)}")
        if labels.shape[0] != images_u8.shape[0]:
            raise ValueError("images and labels differ in length")
        self.device = torch.device(device)
        self.images_u8 = images_u8.contiguous().to(self.device)
        self.labels = labels.to(torch.int64).to(self.device)

    def __len__(self) -> int:
        return self.images_u8.shape[0]

    def gather(self, idx: torch.Tensor):
        """GPU: ``(bf16 [B,H,W,4] NHWC4, int64 [B])``; CPU: ``(float32 [B,3,H,W], int64 [B])``."""
        y = self.labels.index_select(0, idx)
        if self.device.type == "cuda":
            from .. import native

            n, h, w, _ = self.images_u8.shape
            out = torch.empty(idx.numel(), h, w, 4, dtype=torch.bfloat16, device=self.device)
            native.require().image_gather_nhwc4(self.images_u8, idx, out)
            return out, y
        x = self.images_u8.index_select(0, idx).permute(0, 3, 1, 2).float().div_(255.0)
        return x, y


class DeviceImageLoader:
    """The rank's ``DistributedSampler``-exact batches out of device memory (ragged last
    batch, drop_last=False), one index upload per epoch."""

    def __init__(self, data: DeviceImages, batch_size: int, world_size: int, rank: int,
                 shuffle: bool = True, seed: int = 0):
        self.data, self.batch_size = data, int(batch_size)
        self.sampler = ShardedSampler(len(data), world_size, rank, shuffle=shuffle, seed=seed)

    def __len__(self) -> int:
        return steps_per_epoch(len(self.data), self.sampler.num_replicas, self.batch_size)

    def __iter__(self):
        idx = self.sampler.indices().to(self.data.device, non_blocking=False)
        for s in range(0, idx.numel(), self.batch_size):
            yield self.data.gather(idx[s:s + self.batch_size])
