"""BASELINE config 5 plumbing on CPU/gloo: `train_ddp.py --model resnet18` trains ResNet-18
on synthetic ImageNet-shaped data with the reference's DDP loop, rank-0 checkpoints in
torchvision's state_dict layout (OIHW conv weights, BN buffers incl. num_batches_tracked),
and a re-run resumes on both ranks with identical state."""
import os

import torch
import torch.multiprocessing as mp

from ddp_amd.data import DeviceImageLoader, DeviceImages, synthetic_imagenet
from ddp_amd.parallel import free_port


def _worker(rank, ws, port, ckdir, epochs, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from ddp_amd.engine.trainer import TrainOptions, ddp_train

    opts = TrainOptions(backend="gloo", checkpoint_dir=ckdir, log_every=2, model="resnet18",
                        image_size=32, num_classes=10, dataset_size=48, momentum=0.9)
    model = ddp_train(rank, ws, epochs, 8, opts)
    # parameters agree bitwise; BN running stats are rank-local between forwards (torch DDP
    # semantics: broadcast_buffers syncs them from rank 0 at the start of each forward)
    q.put((rank, float(sum(p.double().sum() for p in model.parameters()))))


def test_resnet18_trainer_save_resume_ws2(tmp_path, capfd):
    ck = str(tmp_path / "checkpoints")
    q = mp.get_context("spawn").Queue()
    mp.start_processes(_worker, args=(2, free_port(), ck, 1, q), nprocs=2, start_method="spawn", join=True)
    d = dict(q.get() for _ in range(2))
    assert d[0] == d[1], "ranks diverged"
    out = capfd.readouterr().out
    assert "Epoch 0 | Batch 0 | Loss:" in out and "Rank 1: Starting epoch 0" in out
    ck0 = torch.load(os.path.join(ck, "epoch_0.pt"), weights_only=True)
    m = ck0["model"]
    assert tuple(m["conv1.weight"].shape) == (64, 3, 7, 7)                 # torchvision OIHW
    assert tuple(m["layer2.0.downsample.0.weight"].shape) == (128, 64, 1, 1)
    assert tuple(m["fc.weight"].shape) == (10, 512)
    assert int(m["bn1.num_batches_tracked"]) == 3                       # 48 / 2 ranks / 8 = 3 steps
    assert len(ck0["optimizer"]["state"]) == len([k for k in m if "running" not in k and "num_batches" not in k])
    mp.start_processes(_worker, args=(2, free_port(), ck, 2, q), nprocs=2, start_method="spawn", join=True)
    d = dict(q.get() for _ in range(2))
    assert d[0] == d[1]
    out = capfd.readouterr().out
    assert "Starting epoch 0" not in out and "Rank 1: Starting epoch 1" in out
    assert sorted(os.listdir(ck)) == ["epoch_0.pt", "epoch_1.pt"]
    assert int(torch.load(os.path.join(ck, "epoch_1.pt"), weights_only=True)["model"]["bn1.num_batches_tracked"]) == 6


def test_synthetic_imagenet_loader_shards_like_distributed_sampler():
    imgs, labels = synthetic_imagenet(20, 16, 5, seed=1)
    assert imgs.dtype == torch.uint8 and tuple(imgs.shape) == (20, 16, 16, 3)
    assert int(labels.min()) >= 0 and int(labels.max()) < 5
    d = DeviceImages(imgs, labels, "cpu")
    seen = []
    for r in range(3):
        ld = DeviceImageLoader(d, 3, 3, r)
        ld.sampler.set_epoch(2)
        n = 0
        for x, y in ld:
            assert x.shape[1:] == (3, 16, 16) and x.dtype == torch.float32 and float(x.max()) <= 1.0
            n += x.shape[0]
            seen.append(y)
        assert n == 7  # ceil(20 / 3), padded by wrap-around like DistributedSampler
    assert torch.cat(seen).numel() == 21
