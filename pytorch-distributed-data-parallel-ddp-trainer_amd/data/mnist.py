"""MNIST-shaped training data (reference data.py:11-14).

The reference loads ``torchvision.datasets.MNIST(root="./data", train=True,
transform=ToTensor(), download=True)``: 60,000 uint8 28x28 images, turned into float32
``[1,28,28]`` in [0,1] by ``ToTensor`` (no normalisation), with int labels.  This
environment has neither torchvision nor network access, so:

* ``load_mnist(root, "mnist")`` reads the raw IDX files torchvision leaves under
  ``<root>/MNIST/raw`` (``train-images-idx3-ubyte[.gz]``, ``train-labels-idx1-ubyte[.gz]``)
  with no torchvision dependency;
* ``synthetic_mnist(n)`` produces a deterministic MNIST-shaped set (uint8 pixels in
  [0,255], labels 0-9).  Each class is a smooth 28x28 prototype plus per-image noise, so
  the set is learnable and a training run's loss curve means something.
* ``"auto"`` takes the real files when they exist and the synthetic set otherwise.

Everything stays uint8 until the very last moment: the GPU paths keep the 47 MB uint8
array resident in HBM and apply ``/255`` inside the first convolution.
"""
from __future__ import annotations

import gzip
import os
import struct

import torch

N_TRAIN = 60000
H = W = 28
NUM_CLASSES = 10


def synthetic_mnist(n: int = N_TRAIN, seed: int = 0):
    """Deterministic MNIST-shaped data: ``(uint8 [n,28,28], int64 [n])``."""
    g = torch.Generator().manual_seed(seed)
    labels = torch.randint(0, NUM_CLASSES, (n,), generator=g)
    # smooth class prototypes: 7x7 random fields bilinearly upsampled to 28x28
    coarse = torch.rand(NUM_CLASSES, 1, 7, 7, generator=g)
    protos = torch.nn.functional.interpolate(coarse, size=(H, W), mode="bilinear",
                                             align_corners=False)[:, 0]
    protos = (protos - protos.amin(dim=(1, 2), keepdim=True))
    protos = protos / protos.amax(dim=(1, 2), keepdim=True).clamp_min(1e-6)
    noise = torch.rand(n, H, W, generator=g)
    imgs = (0.65 * protos[labels] + 0.35 * noise) * 255.0
    return imgs.round().clamp_(0, 255).to(torch.uint8), labels


def _open(path: str):
    if os.path.exists(path):
        return open(path, "rb")
    if os.path.exists(path + ".gz"):
        return gzip.open(path + ".gz", "rb")
    raise FileNotFoundError(path)


def read_idx(path: str) -> torch.Tensor:
    """Parse one IDX file (big-endian header: magic = 0x0000 | dtype | ndim, then dims)."""
    with _open(path) as f:
        raw = f.read()
    zero, dtype, ndim = struct.unpack(">HBB", raw[:4])
    if zero != 0 or dtype != 0x08:
        raise ValueError(f"{path}: not an unsigned-byte IDX file (magic {raw[:4].hex()})")
    dims = struct.unpack(">" + "I" * ndim, raw[4:4 + 4 * ndim])
    body = raw[4 + 4 * ndim:]
    count = 1
    for d in dims:
        count *= d
    if len(body) != count:
        raise ValueError(f"{path}: {len(body)} bytes of data, header says {count}")
    return torch.frombuffer(bytearray(body), dtype=torch.uint8).view(*dims)


def _raw_dir(root: str) -> str:
    return os.path.join(root, "MNIST", "raw")


def mnist_available(root: str = "./data") -> bool:
    d = _raw_dir(root)
    return all(os.path.exists(os.path.join(d, f)) or os.path.exists(os.path.join(d, f + ".gz"))
               for f in ("train-images-idx3-ubyte", "train-labels-idx1-ubyte"))


def load_mnist(root: str = "./data", source: str = "auto"):
    """``(uint8 images [N,28,28], int64 labels [N], source_name)``."""
    if source not in ("auto", "mnist", "synthetic"):
        raise ValueError(f"unknown data source {source!r} (auto|mnist|synthetic)")
    if source == "mnist" or (source == "auto" and mnist_available(root)):
        d = _raw_dir(root)
        imgs = read_idx(os.path.join(d, "train-images-idx3-ubyte"))
        labels = read_idx(os.path.join(d, "train-labels-idx1-ubyte")).long()
        if imgs.shape[1:] != (H, W) or imgs.shape[0] != labels.shape[0]:
            raise ValueError(f"unexpected MNIST shapes {tuple(imgs.shape)} / {tuple(labels.shape)}")
        return imgs, labels, "mnist"
    imgs, labels = synthetic_mnist()
    return imgs, labels, "synthetic"


class MNISTDataset(torch.utils.data.Dataset):
    """Map-style dataset with torchvision's ``MNIST(transform=ToTensor())`` item contract:
    ``(float32 [1,28,28] in [0,1], int label)``."""

    def __init__(self, images_u8: torch.Tensor, labels: torch.Tensor):
        self.images = images_u8
        self.labels = labels

    def __len__(self) -> int:
        return self.images.shape[0]

    def __getitem__(self, i):
        return self.images[i].unsqueeze(0).float().div_(255.0), int(self.labels[i])
