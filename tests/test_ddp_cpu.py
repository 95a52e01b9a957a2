"""Multi-process DDP on CPU/gloo (BASELINE config 1)."""
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ddp_amd.models import SimpleCNN, flat_space
from ddp_amd.parallel import bucket_plan, bucket_ranges, free_port


def test_bucket_plan_reproduces_reference_rebuilt_buckets():
    fs = flat_space(SimpleCNN())
    b = bucket_plan(fs)
    # [fl.bias, fl.weight] (2,007,080 B) and [net.2.*, net.0.*] (75,264 B)
    assert b == [["fl.bias", "fl.weight"], ["net.2.bias", "net.2.weight", "net.0.bias", "net.0.weight"]]
    sizes = [sum(fs.numels[n] for n in bk) * 4 for bk in b]
    assert sizes == [2007080, 75264]
    r = bucket_ranges(fs, b)
    assert r[0][0] == 0 and r[0][0] + r[0][1] == r[1][0] and r[1][0] + r[1][1] == fs.numel


def _worker_ddp_equivalence(rank, ws, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    from torch.nn.parallel import DistributedDataParallel as TorchDDP

    from ddp_amd.models import reference_simple_cnn
    from ddp_amd.ops import FusedSGD
    from ddp_amd.parallel import DistributedDataParallel

    torch.manual_seed(100 + rank)  # different init per rank: DDP must broadcast rank 0's
    ours = SimpleCNN()
    ref = reference_simple_cnn()
    torch.manual_seed(7)
    if rank == 0:
        ours_sd = ours.state_dict()
        ref.load_state_dict(ours_sd)
    ddp = DistributedDataParallel(ours)
    tddp = TorchDDP(ref)
    g = torch.Generator().manual_seed(rank)
    x = torch.rand(6, 1, 28, 28, generator=g)
    y = torch.randint(0, 10, (6,), generator=g)
    opt = FusedSGD(ours, lr=0.1)
    topt = torch.optim.SGD(ref.parameters(), lr=0.1)
    for _ in range(2):
        opt.zero_grad()
        topt.zero_grad()
        torch.nn.functional.cross_entropy(ddp(x), y).backward()
        torch.nn.functional.cross_entropy(tddp(x), y).backward()
        opt.step()
        topt.step()
    sd_ours, sd_ref = ours.state_dict(), ref.state_dict()
    err = max((sd_ours[k] - sd_ref[k]).abs().max().item() for k in sd_ref)
    q.put((rank, err, ddp.allreduce_buckets_launched))
    dist.destroy_process_group()


@pytest.mark.slow
@pytest.mark.parametrize("ws", [2, 3, 8])
def test_ddp_matches_torch_ddp_gloo(ws):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    mp.start_processes(_worker_ddp_equivalence, args=(ws, free_port(), q), nprocs=ws,
                       start_method="spawn", join=True)
    res = sorted(q.get() for _ in range(ws))
    for rank, err, launched in res:
        assert err < 1e-5, f"rank {rank} diverges from torch DDP by {err}"
        assert launched == 4  # 2 buckets x 2 iterations


def _worker_train(rank, ws, port, ckdir, epochs, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from ddp_amd.engine.trainer import TrainOptions, ddp_train

    opts = TrainOptions(backend="gloo", checkpoint_dir=ckdir, max_steps=20, num_workers=0,
                        log_every=10, data="synthetic")
    m = ddp_train(rank, ws, epochs, 64, opts)
    import hashlib

    h = hashlib.sha256()
    for p in m.parameters():
        h.update(p.detach().contiguous().numpy().tobytes())
    q.put((rank, h.hexdigest()))  # small payload: a big one deadlocks the join


@pytest.mark.slow
def test_train_save_and_resume_ws2(tmp_path, capfd):
    ck = str(tmp_path / "checkpoints")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    mp.start_processes(_worker_train, args=(2, free_port(), ck, 1, q), nprocs=2,
                       start_method="spawn", join=True)
    digests = dict(q.get() for _ in range(2))
    assert digests[0] == digests[1], "ranks diverged"
    assert sorted(os.listdir(ck)) == ["epoch_0.pt"]
    out = capfd.readouterr().out
    for line in ["Rank: 0 has initialized its process group with world size 2", "Rank 1 initialized",
                 "Rank 0 model wrapped in DDP", "Rank 1: Dataloader ready",
                 "Rank 0: Loss and Optimizer ready", "Rank 0: No checkpoint found, starting from scratch.",
                 "Rank 1: Starting epoch 0", "Epoch 0 | Batch 0 | Loss:", "Epoch 0 | Batch 10 | Loss:",
                 "Rank 1 cleaned up."]:
        assert line in out, line
    assert "Epoch 0 | Batch 0" in out and out.count("| Batch 0 |") == 1  # rank 0 only
    # resume: a re-run with --epochs 2 starts at epoch 1 on BOTH ranks (broken in the reference)
    mp.start_processes(_worker_train, args=(2, free_port(), ck, 2, q), nprocs=2,
                       start_method="spawn", join=True)
    _ = [q.get() for _ in range(2)]
    out = capfd.readouterr().out
    assert "Starting epoch 0" not in out
    assert "Rank 0: Starting epoch 1" in out and "Rank 1: Starting epoch 1" in out
    assert sorted(os.listdir(ck)) == ["epoch_0.pt", "epoch_1.pt"]
    ck1 = torch.load(os.path.join(ck, "epoch_1.pt"), weights_only=True)
    assert ck1["epoch"] == 1


def _worker_fault(rank, ws, port, ckdir, epochs, fault, momentum=0.0):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from ddp_amd.engine.trainer import TrainOptions, ddp_train

    opts = TrainOptions(backend="gloo", checkpoint_dir=ckdir, max_steps=12, num_workers=0,
                        log_every=1000, data="synthetic", fault=fault, momentum=momentum)
    ddp_train(rank, ws, epochs, 32, opts)


@pytest.mark.slow
@pytest.mark.parametrize("momentum", [0.0, 0.9])
def test_fault_then_resume_is_byte_identical(tmp_path, momentum):
    """BASELINE config 4 on CPU/gloo: crash mid-epoch, auto-resume, final checkpoint equals
    the uninterrupted run's (every zip record except the random serialization_id) - with
    momentum the resumed ranks (rank 0 loads, rank 1 receives the broadcast) continue the
    momentum buffer instead of re-initialising it."""
    import zipfile

    a, b = str(tmp_path / "a"), str(tmp_path / "b")
    mp.start_processes(_worker_fault, args=(2, free_port(), a, 3, None, momentum), nprocs=2,
                       start_method="spawn", join=True)
    with pytest.raises(Exception):
        mp.start_processes(_worker_fault, args=(2, free_port(), b, 3, (1, 5, 1), momentum), nprocs=2,
                           start_method="spawn", join=True)
    assert sorted(os.listdir(b)) == ["epoch_0.pt"]
    mp.start_processes(_worker_fault, args=(2, free_port(), b, 3, None, momentum), nprocs=2,
                       start_method="spawn", join=True)
    za, zb = zipfile.ZipFile(os.path.join(a, "epoch_2.pt")), zipfile.ZipFile(os.path.join(b, "epoch_2.pt"))
    diff = [i.filename for i in za.infolist() if za.read(i.filename) != zb.read(i.filename)]
    assert set(diff) <= {"epoch_2/.data/serialization_id"}, diff


@pytest.mark.slow
def test_cli_under_torchrun_2proc(tmp_path):
    """BASELINE config 1: `torchrun --nproc_per_node=2 train_ddp.py` on CPU/gloo.  Exactly 2
    trainer ranks (no nested self-spawn, reference bug B3), a checkpoint, clean exit."""
    import subprocess
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(repo, "train_ddp.py"), "--epochs", "1", "--batch_size", "64",
           "--max_steps", "15", "--num_workers", "0", "--data", "synthetic", "--log_every", "5"]
    p = subprocess.run(cmd, cwd=tmp_path, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    out = p.stdout
    assert out.count("has initialized its process group with world size 2") == 2
    assert "Rank 0 initialized" in out and "Rank 1 initialized" in out and "Rank 2" not in out
    assert "Epoch 0 | Batch 10 | Loss:" in out
    assert os.path.exists(tmp_path / "checkpoints" / "epoch_0.pt")


def test_grad_accum_matches_large_batch(tmp_path):
    """--grad_accum 2 at batch 16 == one step at batch 32 (same samples, mean loss)."""
    from ddp_amd.engine.trainer import TrainOptions, ddp_train

    def run(bs, accum, sub):
        o = TrainOptions(backend="gloo", data="synthetic", save=False, num_workers=0,
                         max_steps=8 * accum, checkpoint_dir=str(tmp_path / sub), grad_accum=accum,
                         log_every=1000)
        return ddp_train(0, 1, 1, bs, o)

    m1 = run(32, 1, "a")
    m2 = run(16, 2, "b")
    for (n, a), (_, b) in zip(m1.named_parameters(), m2.named_parameters()):
        assert torch.allclose(a, b, rtol=1e-4, atol=1e-6), n


def _worker_bf16_copy_after_broadcast(rank, ws, port, q):
    """A c10d broadcast into the flat parameters does not bump their version counter: the
    bf16 weight copy the MFMA kernels read must still be rebuilt (the r3 multi-rank GPU
    rehearsal found a resumed rank 1 training on its own stale init through that copy)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    from ddp_amd.ops import FusedSGD
    from ddp_amd.parallel import DistributedDataParallel
    from ddp_amd.utils.checkpoint import resume

    torch.manual_seed(100 + rank)  # different init per rank
    m = SimpleCNN()
    fs = flat_space(m)
    stale = fs.bf16_params().clone()  # built from this rank's own init
    DistributedDataParallel(m)        # construction: rank 0's parameters broadcast
    ok_ctor = torch.equal(fs.bf16_params(), fs.params.to(torch.bfloat16))
    # resume() broadcasts the flat buffer the same way
    ck = os.environ["DDP_AMD_TEST_CKDIR"]
    opt = FusedSGD(m, lr=0.1)
    fs.bf16_params()
    resume(m, opt, ck, rank, ws, flat=fs)
    ok_resume = torch.equal(fs.bf16_params(), fs.params.to(torch.bfloat16))
    q.put((rank, ok_ctor, ok_resume, rank == 0 or not torch.equal(stale, fs.bf16_params())))
    dist.destroy_process_group()


def test_bf16_copy_rebuilt_after_broadcasts(tmp_path):
    from ddp_amd.ops import FusedSGD
    from ddp_amd.utils.checkpoint import save_checkpoint

    torch.manual_seed(5)
    m = SimpleCNN()
    save_checkpoint(str(tmp_path), 0, m, FusedSGD(m, lr=0.1))
    os.environ["DDP_AMD_TEST_CKDIR"] = str(tmp_path)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_worker_bf16_copy_after_broadcast, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert all(r[1] and r[2] and r[3] for r in res), res
