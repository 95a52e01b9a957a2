"""Shape-only multi-rank checks on torch's fake process group.

One process pretends to be rank r of an 8-rank job: every collective returns
immediately, so the *sequence* of collectives our DDP issues (construction sync,
per-step bucket all-reduces) can be checked against the reference's implicit DDP
sequence at world sizes no CPU box could run for real.
"""
import pytest
import torch
import torch.distributed as dist

fake_pg = pytest.importorskip("torch.testing._internal.distributed.fake_pg")


@pytest.fixture
def fake_world(request):
    rank, ws = request.param
    dist.init_process_group("fake", store=fake_pg.FakeStore(), rank=rank, world_size=ws)
    yield rank, ws
    dist.destroy_process_group()


@pytest.mark.parametrize("fake_world", [(0, 8), (5, 8), (1, 4)], indirect=True)
def test_ddp_collective_sequence_matches_reference_buckets(fake_world):
    from ddp_amd.models import SimpleCNN
    from ddp_amd.parallel import DistributedDataParallel
    from ddp_amd.utils.debug import CollectiveTracer

    rank, ws = fake_world
    torch.manual_seed(0)
    with CollectiveTracer() as tr:
        ddp = DistributedDataParallel(SimpleCNN())
        ctor = list(tr.log)
        x = torch.rand(4, 1, 28, 28)
        y = torch.randint(0, 10, (4,))
        for _ in range(2):
            torch.nn.functional.cross_entropy(ddp(x), y).backward()
        steps = tr.log[len(ctor):]
    # construction: metadata check, then ONE broadcast of the flat parameter buffer from rank 0
    bcasts = [e for e in ctor if e[0] == "broadcast"]
    assert bcasts and bcasts[-1][2] == 0
    assert bcasts[-1][1][1][0] >= 520_586
    # every step: exactly the reference's two rebuilt buckets, fc first (I6, I7)
    # (our flat buckets hold each parameter 64-element aligned, so a bucket carries the
    # reference's element count plus < 64 zero-pad elements per parameter)
    ar = [e for e in steps if e[0] == "all_reduce"]
    assert len(ar) == 4
    for e, (want, nparam) in zip(ar, [(501_770, 2), (18_816, 4)] * 2):
        assert e[1][0] == "torch.float32"
        assert want <= e[1][1][0] < want + 64 * nparam
    # gradients were prescaled by 1/ws (fake all-reduce leaves the local SUM contribution)
    assert ddp.fs.grads.abs().sum() > 0


@pytest.mark.parametrize("fake_world", [(3, 8)], indirect=True)
def test_no_sync_skips_allreduce(fake_world):
    from ddp_amd.models import SimpleCNN
    from ddp_amd.parallel import DistributedDataParallel
    from ddp_amd.utils.debug import CollectiveTracer

    ddp = DistributedDataParallel(SimpleCNN())
    x = torch.rand(2, 1, 28, 28)
    y = torch.randint(0, 10, (2,))
    with CollectiveTracer() as tr:
        with ddp.no_sync():
            torch.nn.functional.cross_entropy(ddp(x), y).backward()
        n_nosync = sum(1 for e in tr.log if e[0] == "all_reduce")
        torch.nn.functional.cross_entropy(ddp(x), y).backward()
        n_sync = sum(1 for e in tr.log if e[0] == "all_reduce")
    assert n_nosync == 0 and n_sync == 2


@pytest.mark.parametrize("fake_world", [(2, 8)], indirect=True)
def test_broadcast_buffers_one_collective_per_dtype(fake_world):
    """``broadcast_buffers=True`` (the reference's DDP default) costs one flat broadcast per
    buffer DTYPE per forward for ResNet-18's 60 BatchNorm buffers (float32 running stats,
    int64 num_batches_tracked: 2; torch DDP coalesces likewise), and the BN kernels'
    in-place running-stat updates land in the flat tensors."""
    from ddp_amd.models import resnet18
    from ddp_amd.parallel import DistributedDataParallel
    from ddp_amd.utils.debug import CollectiveTracer

    torch.manual_seed(0)
    model = resnet18(num_classes=10)
    nbuf = sum(1 for _ in model.buffers())
    assert nbuf == 60
    with CollectiveTracer() as tr:
        ddp = DistributedDataParallel(model)
        ctor = len(tr.log)
        x = torch.randn(2, 3, 32, 32)
        for _ in range(3):
            ddp(x).sum().backward()
        steps = tr.log[ctor:]
    bc = [e for e in steps if e[0] == "broadcast"]
    assert len(bc) == 6 and ddp.buffer_broadcasts == 3
    assert sorted({e[1][0] for e in bc}) == ["torch.float32", "torch.int64"] and all(e[2] == 0 for e in bc)
    flats = {t.dtype: t for t in ddp.bufs.flat_list()}
    for dt in (torch.float32, torch.int64):
        total = sum(b.numel() for b in model.buffers() if b.dtype == dt)
        assert flats[dt].numel() >= total
    # every buffer is a view of its dtype's flat tensor; running stats moved off their init values
    def inside(b):
        f = flats[b.dtype]
        return f.data_ptr() <= b.data_ptr() < f.data_ptr() + f.numel() * f.element_size()
    assert all(inside(b) for b in model.buffers())
    bn = model.bn1
    assert int(bn.num_batches_tracked) == 3 and bn.running_mean.abs().sum() > 0
    # a buffer replaced by a new tensor is pulled back into the flat tensor before the next broadcast
    bn.running_var = torch.full_like(bn.running_var, 2.0)
    ddp(x)
    assert inside(bn.running_var) and 1.5 < float(bn.running_var[0]) < 2.0  # 0.9 * 2 + 0.1 * var


def test_buffer_space_state_dict_saves_and_reassigns(tmp_path):
    """with every buffer in ONE byte storage, torch.save of a BatchNorm model's
    state_dict refused ("view the same data as different types").  Per-dtype flat tensors:
    the reference-style save works, the saved values round-trip, buffer reassignment is
    pulled back, BN train-mode backward still works after in-place stat updates, and a
    dtype change (.double()) rebuilds the space instead of being copied back."""
    import torch.nn as nn

    from ddp_amd.models.layers import buffer_space

    torch.manual_seed(0)
    m = nn.Sequential(nn.Conv2d(3, 8, 3, padding=1), nn.BatchNorm2d(8), nn.ReLU(), nn.Conv2d(8, 4, 1),
                      nn.BatchNorm2d(4))
    bs = buffer_space(m)
    assert len(bs.flat_list()) == 2
    x = torch.randn(4, 3, 8, 8)
    for _ in range(2):  # BN backward after in-place running-stat updates (own version counters)
        m(x).square().mean().backward()
    assert int(m[1].num_batches_tracked) == 2
    path = tmp_path / "sd.pt"
    torch.save(m.state_dict(), path)  # the reference's save pattern (train_ddp.py:205-209)
    sd = torch.load(path, weights_only=True)
    for k, v in m.state_dict().items():
        assert torch.equal(sd[k], v), k
    # reassignment then forward: pulled back into the flat tensor
    m[1].running_mean = torch.full_like(m[1].running_mean, 3.0)
    bs2 = buffer_space(m)
    assert bs2 is bs and float(m[1].running_mean[0]) == 3.0
    f32 = bs.flats[torch.float32]
    assert f32.data_ptr() <= m[1].running_mean.data_ptr() < f32.data_ptr() + f32.numel() * 4
    # a dtype change rebuilds instead of silently casting back to float32
    m.double()
    bs3 = buffer_space(m)
    assert bs3 is not bs and m[1].running_mean.dtype == torch.float64
    assert float(m[1].running_mean[0]) == 3.0
    m(x.double()).sum().backward()
    torch.save(m.state_dict(), tmp_path / "sd64.pt")
