"""Checkpoint contract: byte-compatible saves, robust discovery."""
import os
import time
import zipfile

import pytest
import torch

from ddp_amd.models import SimpleCNN, reference_simple_cnn
from ddp_amd.ops import FusedSGD
from ddp_amd.utils import discover_latest, load_checkpoint, save_checkpoint

REF = "/root/reference/checkpoints"
needs_ref = pytest.mark.skipif(not os.path.isdir(REF), reason="reference checkout not mounted")


@needs_ref
@pytest.mark.parametrize("epoch", [0, 1])
def test_resave_reference_checkpoint_is_byte_identical(tmp_path, epoch):
    ref = os.path.join(REF, f"epoch_{epoch}.pt")
    ck = load_checkpoint(ref)
    assert ck["epoch"] == epoch
    m = SimpleCNN()
    m.load_state_dict(ck["model"])
    out = save_checkpoint(tmp_path, ck["epoch"], m, FusedSGD(m, lr=0.01))
    a, b = zipfile.ZipFile(ref), zipfile.ZipFile(out)
    assert [i.filename for i in a.infolist()] == [i.filename for i in b.infolist()]
    diff = [i.filename for i in a.infolist() if a.read(i.filename) != b.read(i.filename)]
    assert diff == [f"epoch_{epoch}/.data/serialization_id"]
    assert os.path.getsize(ref) == os.path.getsize(out)


def test_schema_matches_stock_torch_objects(tmp_path):
    torch.manual_seed(3)
    ours = SimpleCNN()
    torch.manual_seed(3)
    ref = reference_simple_cnn()
    opt_ref = torch.optim.SGD(ref.parameters(), lr=0.01)
    p = save_checkpoint(tmp_path, 4, ours, FusedSGD(ours, lr=0.01))
    ck = load_checkpoint(p)
    assert ck["epoch"] == 4
    assert list(ck["model"].keys()) == list(ref.state_dict().keys())
    assert ck["model"]._metadata == ref.state_dict()._metadata
    for k, v in ref.state_dict().items():
        assert torch.equal(ck["model"][k], v)
        assert ck["model"][k].stride() == v.stride()
    assert ck["optimizer"] == opt_ref.state_dict()


def test_state_roundtrip_with_momentum(tmp_path):
    torch.manual_seed(0)
    m = SimpleCNN()
    opt = FusedSGD(m, lr=0.05, momentum=0.9)
    x, y = torch.rand(4, 1, 28, 28), torch.randint(0, 10, (4,))
    for _ in range(2):
        opt.zero_grad()
        torch.nn.functional.cross_entropy(m(x), y).backward()
        opt.step()
    p = save_checkpoint(tmp_path, 0, m, opt)
    ck = load_checkpoint(p)
    # momentum buffers are stored in the reference layout, like torch.optim.SGD would
    assert ck["optimizer"]["state"][2]["momentum_buffer"].shape == (64, 32, 3, 3)
    m2 = SimpleCNN()
    o2 = FusedSGD(m2, lr=0.0)
    m2.load_state_dict(ck["model"])
    o2.load_state_dict(ck["optimizer"])
    assert o2.param_groups[0]["lr"] == 0.05
    assert torch.equal(o2.momentum_buffer, opt.momentum_buffer)
    for a, b in zip(m.parameters(), m2.parameters()):
        assert torch.equal(a, b)


def test_discovery_newest_by_ctime_with_epoch_tiebreak(tmp_path):
    d = tmp_path / "checkpoints"
    assert discover_latest(d) is None and d.exists()  # created like the reference's mkdir
    for e in (0, 1, 2):
        (d / f"epoch_{e}.pt").write_bytes(b"x")
    (d / "notes.txt").write_text("ignored")
    # identical ctimes can happen (the reference's mounted files do): epoch number breaks ties
    assert discover_latest(d).name == "epoch_2.pt"
    time.sleep(0.02)
    os.utime(d / "epoch_0.pt")
    (d / "epoch_0.pt").write_bytes(b"y")  # rewrite -> newest ctime wins
    assert discover_latest(d).name == "epoch_0.pt"


def test_atomic_save_leaves_no_temp(tmp_path):
    m = SimpleCNN()
    save_checkpoint(tmp_path, 7, m, FusedSGD(m, lr=0.01))
    assert sorted(os.listdir(tmp_path)) == ["epoch_7.pt"]
