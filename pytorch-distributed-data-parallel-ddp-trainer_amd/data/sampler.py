"""DistributedSampler-exact per-rank index lists (reference data.py:16-19).

The reference shards MNIST with ``DistributedSampler(dataset, num_replicas=ws, rank=r,
shuffle=True)`` (seed 0, drop_last False).  Its index math
(torch/utils/data/distributed.py:98-141) is reproduced here as whole-tensor ops instead
of Python lists: one CPU ``randperm`` seeded with ``seed + epoch`` (the CPU generator, so
the permutation is the same one torch's sampler draws), wrap-around padding to
``ceil(N/ws)*ws`` and a strided slice ``[rank::ws]``.  The result is an int64 tensor
that the device loader uploads once per epoch (240 KB at ws=1) instead of shipping
indices batch by batch.
"""
from __future__ import annotations

import math

import torch


def num_samples(n: int, world_size: int, drop_last: bool = False) -> int:
    """Per-rank sample count (torch/utils/data/distributed.py:95-103)."""
    if drop_last and n % world_size != 0:
        return math.ceil((n - world_size) / world_size)
    return math.ceil(n / world_size)


def steps_per_epoch(n: int, world_size: int, batch_size: int, drop_last: bool = False) -> int:
    """DataLoader length for the rank's shard (the loader itself keeps ragged batches)."""
    return math.ceil(num_samples(n, world_size, drop_last) / batch_size)


def epoch_indices(n: int, world_size: int, rank: int, epoch: int, shuffle: bool = True,
                  seed: int = 0, drop_last: bool = False) -> torch.Tensor:
    """The indices ``DistributedSampler`` yields for ``rank`` in ``epoch`` (int64)."""
    if not 0 <= rank < world_size:
        raise ValueError(f"Invalid rank {rank}, rank should be in the interval [0, {world_size - 1}]")
    if shuffle:
        g = torch.Generator()
        g.manual_seed(seed + epoch)
        idx = torch.randperm(n, generator=g)
    else:
        idx = torch.arange(n)
    total = num_samples(n, world_size, drop_last) * world_size
    # wrap-around padding (indices + indices[:pad], repeated when pad > n) is a periodic
    # extension of the permutation, i.e. a prefix of repeat(); drop_last is a truncation
    idx = idx.repeat(math.ceil(total / n))[:total] if total > n else idx[:total]
    return idx[rank:total:world_size].clone()


class ShardedSampler(torch.utils.data.Sampler):
    """Drop-in ``DistributedSampler`` replacement that also hands out the whole epoch as
    one tensor (``indices()``), which the HBM-resident loader and the fused engine use."""

    def __init__(self, n: int, num_replicas: int, rank: int, shuffle: bool = True,
                 seed: int = 0, drop_last: bool = False):
        if not 0 <= rank < num_replicas:
            raise ValueError(f"Invalid rank {rank}, rank should be in the interval [0, {num_replicas - 1}]")
        self.n = int(n)
        self.num_replicas, self.rank = int(num_replicas), int(rank)
        self.shuffle, self.seed, self.drop_last = shuffle, int(seed), drop_last
        self.epoch = 0
        self.num_samples = num_samples(self.n, self.num_replicas, drop_last)
        self.total_size = self.num_samples * self.num_replicas

    def set_epoch(self, epoch: int) -> None:
        self.epoch = int(epoch)

    def indices(self) -> torch.Tensor:
        return epoch_indices(self.n, self.num_replicas, self.rank, self.epoch, self.shuffle,
                             self.seed, self.drop_last)

    def __iter__(self):
        return iter(self.indices().tolist())

    def __len__(self) -> int:
        return self.num_samples
