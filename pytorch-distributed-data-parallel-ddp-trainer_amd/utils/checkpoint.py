"""Checkpoint save / discovery / resume (reference train_ddp.py:45-185 and 204-209).

On-disk contract (unchanged): ``./checkpoints/epoch_{epoch}.pt``
written by rank 0 after every epoch with
``torch.save({"epoch", "model": model.module.state_dict(), "optimizer": opt.state_dict()})``,
CPU fp32 tensors, no ``module.`` prefix.  Because the dict is built exactly like
the reference's (same key order, ``OrderedDict`` + ``_metadata``, SGD
``param_groups`` keys) ``torch.save`` reproduces the reference's bytes except the
random ``.data/serialization_id`` record (tests/test_checkpoint.py compares every
zip record with the reference's own ``epoch_0.pt``).

Fixes of the reference's resume path:
* B6/B7/B8/B9 - the 33-broadcast per-key protocol (broken as shipped) is replaced
  by: rank 0 loads with ``weights_only=True``, then ONE broadcast of the epoch,
  ONE broadcast of the flat parameter buffer (any dtype), ONE of the optimizer
  state (momentum buffer) and the hyper-parameters;
* B10 - the optimizer state is applied, not just read;
* B11 - only ``*.pt`` files are candidates; newest by ``st_ctime`` with ties
  broken by the parsed epoch number (the reference picked by directory order);
* B13 - the save is atomic (temp directory + ``os.replace``, keeping the
  archive-internal name ``epoch_N`` that ``torch.save`` derives from the file
  name) and followed by a barrier.
"""
from __future__ import annotations

import os
import re
import shutil
import uuid
from pathlib import Path

import torch
import torch.distributed as dist

_EPOCH_RE = re.compile(r"epoch_(\d+)\.pt$")


def checkpoint_path(ckpt_dir: str | os.PathLike, epoch: int) -> str:
    return os.path.join(str(ckpt_dir), f"epoch_{epoch}.pt")


def _epoch_of(p: Path) -> int:
    m = _EPOCH_RE.search(p.name)
    return int(m.group(1)) if m else -1


def discover_latest(ckpt_dir: str | os.PathLike = "./checkpoints", create: bool = True):
    """Newest checkpoint in ``ckpt_dir`` (or None).  Creates the directory if missing."""
    d = Path(ckpt_dir)
    if not d.exists():
        if create:
            d.mkdir(parents=True, exist_ok=True)
        return None
    files = [f for f in d.iterdir() if f.is_file() and f.suffix == ".pt"]
    if not files:
        return None
    return max(files, key=lambda f: (f.stat().st_ctime, _epoch_of(f), f.name))


def build_checkpoint(epoch: int, model: torch.nn.Module, optimizer) -> dict:
    """The reference's checkpoint dict, with CPU tensors (key order matters for the bytes)."""
    sd = model.state_dict()
    cpu_sd = type(sd)()
    for k, v in sd.items():
        cpu_sd[k] = v.detach().to("cpu").clone(memory_format=torch.contiguous_format)
    cpu_sd._metadata = getattr(sd, "_metadata", None)
    if cpu_sd._metadata is None:
        del cpu_sd._metadata
    osd = optimizer.state_dict()
    for s in osd.get("state", {}).values():
        for k, v in list(s.items()):
            if torch.is_tensor(v):
                s[k] = v.detach().to("cpu").clone(memory_format=torch.contiguous_format)
    return {"epoch": epoch, "model": cpu_sd, "optimizer": osd}


def save_checkpoint(ckpt_dir, epoch: int, model, optimizer) -> str:
    """Atomically write ``ckpt_dir/epoch_{epoch}.pt`` (call on rank 0 only)."""
    os.makedirs(ckpt_dir, exist_ok=True)
    final = checkpoint_path(ckpt_dir, epoch)
    tmpdir = os.path.join(str(ckpt_dir), f".tmp-{uuid.uuid4().hex[:8]}")
    os.makedirs(tmpdir)
    try:
        tmp = os.path.join(tmpdir, os.path.basename(final))  # same basename -> same archive name
        torch.save(build_checkpoint(epoch, model, optimizer), tmp)
        os.replace(tmp, final)
    finally:
        shutil.rmtree(tmpdir, ignore_errors=True)
    return final


def load_checkpoint(path) -> dict:
    """Safe load (never unpickles arbitrary objects)."""
    return torch.load(str(path), map_location="cpu", weights_only=True)


def resume(model, optimizer, ckpt_dir="./checkpoints", rank: int = 0, world_size: int = 1,
           device=None, flat=None) -> tuple[int, str | None]:
    """Collective: discover on rank 0, load, and make every rank's state identical.

    Returns ``(start_epoch, path or None)``.  ``flat`` is the model's FlatSpace (so
    parameters travel in one broadcast); ``device`` is where broadcasts happen
    (cuda for RCCL, cpu for gloo).
    """
    dist_on = world_size > 1 and dist.is_initialized()
    bdev = device if device is not None else torch.device("cpu")
    flag = torch.zeros(2, dtype=torch.int64, device=bdev)  # [found, start_epoch]
    latest = None
    ckpt = None
    if rank == 0:
        latest = discover_latest(ckpt_dir, create=True)
        if latest is not None:
            ckpt = load_checkpoint(latest)
            model.load_state_dict(ckpt["model"])
            optimizer.load_state_dict(ckpt["optimizer"])
            flag[0] = 1
            flag[1] = int(ckpt["epoch"]) + 1
    if dist_on:
        dist.broadcast(flag, src=0)
        dist.barrier()  # checkpoint folder exists for everyone (reference train_ddp.py:63)
    if int(flag[0]) == 0:
        return 0, None
    if dist_on:
        with torch.no_grad():
            if flat is not None:
                dist.broadcast(flat.params, src=0)
                flat.params_written()  # (the broadcast does not bump the version counter)
            else:
                for p in model.parameters():
                    dist.broadcast(p.data, src=0)
            from ..models.layers import buffer_space

            bs = buffer_space(model)  # every buffer: one flat broadcast per dtype
            if bs is not None:
                for t in bs.flat_list():
                    dist.broadcast(t, src=0)
        hp = [optimizer.param_groups[0] if rank == 0 else None]
        dist.broadcast_object_list(hp, src=0)
        optimizer.param_groups[0].update(hp[0])
        has_mom = torch.tensor([1 if getattr(optimizer, "momentum_buffer", None) is not None else 0],
                               device=bdev)
        dist.broadcast(has_mom, src=0)
        if int(has_mom) == 1:
            if optimizer.momentum_buffer is None:
                optimizer.momentum_buffer = torch.zeros_like(flat.params)
            dist.broadcast(optimizer.momentum_buffer, src=0)
            if hasattr(optimizer, "mark_started"):
                optimizer.mark_started()
    return int(flag[1]), (str(latest) if latest is not None else "(broadcast from rank 0)")
