"""Data layer (reference data.py:6-27): IDX reader, synthetic set, get_dataloader contract."""
import gzip
import struct

import pytest
import torch
from torch.utils.data import DataLoader, DistributedSampler

from ddp_amd.data import (MNISTDataset, get_dataloader, load_mnist, mnist_available, read_idx,
                          synthetic_mnist)


def _write_idx(path, t: torch.Tensor, gz=False):
    hdr = struct.pack(">HBB", 0, 0x08, t.dim()) + struct.pack(">" + "I" * t.dim(), *t.shape)
    data = hdr + t.contiguous().numpy().tobytes()
    if gz:
        with gzip.open(str(path) + ".gz", "wb") as f:
            f.write(data)
    else:
        path.write_bytes(data)


@pytest.mark.parametrize("gz", [False, True])
def test_idx_roundtrip_and_auto_source(tmp_path, gz):
    raw = tmp_path / "MNIST" / "raw"
    raw.mkdir(parents=True)
    imgs = torch.randint(0, 256, (50, 28, 28), dtype=torch.uint8)
    labels = torch.randint(0, 10, (50,), dtype=torch.uint8)
    _write_idx(raw / "train-images-idx3-ubyte", imgs, gz)
    _write_idx(raw / "train-labels-idx1-ubyte", labels, gz)
    assert mnist_available(str(tmp_path))
    assert torch.equal(read_idx(str(raw / "train-images-idx3-ubyte")), imgs)
    x, y, src = load_mnist(str(tmp_path), "auto")
    assert src == "mnist" and torch.equal(x, imgs) and torch.equal(y, labels.long())
    _, _, src = load_mnist(str(tmp_path / "nowhere"), "auto")
    assert src == "synthetic"
    with pytest.raises(FileNotFoundError):
        load_mnist(str(tmp_path / "nowhere"), "mnist")


def test_idx_rejects_bad_files(tmp_path):
    p = tmp_path / "bad"
    p.write_bytes(struct.pack(">HBB", 0, 0x0D, 1) + struct.pack(">I", 4) + b"\0" * 16)
    with pytest.raises(ValueError):
        read_idx(str(p))
    p.write_bytes(struct.pack(">HBB", 0, 0x08, 1) + struct.pack(">I", 9) + b"\0" * 4)
    with pytest.raises(ValueError):
        read_idx(str(p))


def test_synthetic_is_deterministic_mnist_shaped_and_learnable():
    a, la = synthetic_mnist(2000)
    b, lb = synthetic_mnist(2000)
    assert torch.equal(a, b) and torch.equal(la, lb)
    assert a.dtype == torch.uint8 and a.shape == (2000, 28, 28)
    assert la.min() >= 0 and la.max() <= 9 and len(la.unique()) == 10
    # nearest class-mean classifier beats chance by a wide margin -> a learnable set
    x = a.float().view(2000, -1)
    means = torch.stack([x[la == c].mean(0) for c in range(10)])
    pred = torch.cdist(x, means).argmin(1)
    assert (pred == la).float().mean() > 0.5


def test_get_dataloader_matches_reference_loader():
    """Same batches as DataLoader(MNIST, sampler=DistributedSampler(shuffle=True)) including
    the ragged last batch (ws=2, B=32 -> 938 steps with a final batch of 16)."""
    ours, sampler = get_dataloader(32, 2, 1, source="synthetic", num_workers=0)
    imgs, labels, _ = load_mnist(source="synthetic")
    ds = MNISTDataset(imgs, labels)
    ref_sampler = DistributedSampler(ds, num_replicas=2, rank=1, shuffle=True)
    ref = DataLoader(ds, batch_size=32, sampler=ref_sampler)
    assert len(ours) == len(ref) == 938
    for epoch in (0, 3):
        sampler.set_epoch(epoch)
        ref_sampler.set_epoch(epoch)
        it_o, it_r = iter(ours), iter(ref)
        for i in range(3):
            (xo, yo), (xr, yr) = next(it_o), next(it_r)
            assert torch.equal(xo, xr) and torch.equal(yo, yr)
    *_, (xl, yl) = iter(ours)
    assert xl.shape == (16, 1, 28, 28) and yl.dtype == torch.int64
    assert 0.0 <= float(xl.min()) and float(xl.max()) <= 1.0
