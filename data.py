"""Reference-compatible import path: ``from data import get_dataloader`` (reference data.py).

``get_dataloader(batch_size, world_size, rank)`` returns ``(DataLoader, sampler)`` over
MNIST IDX files under ./data if present, else a synthetic MNIST-shaped set (no network
here).  The MI355X training path uses ``ddp_amd.data.DeviceMNISTLoader`` instead
(dataset resident in HBM, gather fused into the first conv kernel).
"""
from ddp_amd.data.loader import get_dataloader  # noqa: F401

__all__ = ["get_dataloader"]
