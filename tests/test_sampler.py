"""ShardedSampler / epoch_indices are bit-exact with torch's DistributedSampler."""
import pytest
import torch
from torch.utils.data import DistributedSampler

from ddp_amd.data import ShardedSampler, epoch_indices, steps_per_epoch


class _Len:
    def __init__(self, n):
        self.n = n

    def __len__(self):
        return self.n


@pytest.mark.parametrize("n", [60000, 1000, 7])
@pytest.mark.parametrize("ws", [1, 2, 3, 4, 8])
def test_matches_torch_distributed_sampler(n, ws):
    for rank in range(ws):
        ref = DistributedSampler(_Len(n), num_replicas=ws, rank=rank, shuffle=True)
        ours = ShardedSampler(n, ws, rank)
        for epoch in (0, 1, 5):
            ref.set_epoch(epoch)
            ours.set_epoch(epoch)
            assert list(ref) == ours.indices().tolist()
            assert len(ref) == len(ours)


@pytest.mark.parametrize("drop_last", [True, False])
def test_drop_last_and_noshuffle(drop_last):
    n, ws = 1003, 4
    for rank in range(ws):
        ref = DistributedSampler(_Len(n), num_replicas=ws, rank=rank, shuffle=False, drop_last=drop_last)
        got = epoch_indices(n, ws, rank, 0, shuffle=False, drop_last=drop_last)
        assert list(ref) == got.tolist()


def test_steps_per_epoch_table():
    # SURVEY §3.4 trip-count table (60,000 samples)
    table = {(1, 32): 1875, (1, 64): 938, (2, 32): 938, (2, 64): 469, (4, 32): 469,
             (4, 64): 235, (8, 32): 235, (8, 64): 118}
    for (ws, b), steps in table.items():
        assert steps_per_epoch(60000, ws, b) == steps


def test_ranks_partition_the_epoch():
    n, ws = 60000, 8
    allidx = torch.cat([epoch_indices(n, ws, r, 3) for r in range(ws)])
    assert allidx.numel() == n
    assert torch.equal(allidx.sort().values, torch.arange(n))
