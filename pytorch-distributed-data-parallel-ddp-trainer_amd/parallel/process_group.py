"""Process-group runtime (reference utils.py:5-19).

``setup(rank, world_size)`` keeps the reference's contract and log line but is
explicit about the transport instead of silently auto-selecting:

* GPU visible -> backend ``"nccl"`` (which *is* RCCL on ROCm) for the c10d
  control plane, the process is bound to its **local** rank's GPU (the
  reference used the global rank, bug B5), and a native RCCL communicator
  (:func:`native_comm`) is bootstrapped over the same TCPStore for the data
  plane (bucket all-reduces issued from C++ on our own HIP streams);
* CPU only -> ``"gloo"`` (the reference's only working configuration, BASELINE
  config 1) - but only when no GPU run was asked for: ``device="gpu"`` (the CLI's
  ``--device gpu``, ``DDP_AMD_DEVICE=gpu``) or a host that exposes a GPU (``/dev/kfd``)
  whose HIP runtime then fails to come up raise instead of quietly training on the CPU
  (the reference's ``utils.py:6`` auto-select would silently fall back to gloo).

``MASTER_ADDR``/``MASTER_PORT`` default to 127.0.0.1 and a free port when unset
(bug B2), and the PG timeout is configurable (``DDP_AMD_PG_TIMEOUT`` seconds).
"""
from __future__ import annotations

import datetime
import os
import socket

import torch
import torch.distributed as dist

_native_comm = None


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def ensure_master_env():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if "MASTER_PORT" not in os.environ:
        os.environ["MASTER_PORT"] = str(free_port())


def local_rank(rank: int | None = None) -> int:
    if "LOCAL_RANK" in os.environ:
        return int(os.environ["LOCAL_RANK"])
    r = rank if rank is not None else int(os.environ.get("RANK", 0))
    n = torch.cuda.device_count() if torch.cuda.is_available() else 1
    return r % max(1, n)


def default_backend() -> str:
    return "nccl" if torch.cuda.is_available() else "gloo"


_VISIBILITY_VARS = ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES")


def _gpu_host() -> bool:
    """The host exposes an AMD GPU (the KFD device node) and the user did not hide every
    device (an empty HIP_ / ROCR_ / CUDA_VISIBLE_DEVICES means "no GPU requested") - a GPU
    run is the expected one."""
    if any(os.environ.get(v, "x") == "" for v in _VISIBILITY_VARS):
        return False
    return os.path.exists("/dev/kfd")


def resolve_backend(backend: str | None = None, device: str | None = None) -> str:
    """The c10d backend for this run, explicit about the transport.

    ``backend``: ``rccl``/``nccl`` | ``gloo`` | None (from ``DDP_AMD_BACKEND`` or the device).
    ``device``: ``gpu`` | ``cpu`` | ``auto``/None (from ``DDP_AMD_DEVICE``).  Raises
    ``RuntimeError`` when a GPU run was requested (``device="gpu"``, ``backend="rccl"``, or
    a GPU host in ``auto`` mode) but no HIP device is usable, instead of silently
    training on the CPU over gloo."""
    backend = backend or os.environ.get("DDP_AMD_BACKEND") or None
    device = (device or os.environ.get("DDP_AMD_DEVICE") or "auto").lower()
    if device not in ("auto", "gpu", "cpu"):
        raise ValueError(f"device must be auto|gpu|cpu, got {device!r}")
    if backend == "rccl":
        backend = "nccl"
    if backend not in (None, "nccl", "gloo"):
        raise ValueError(f"unknown backend {backend!r} (rccl|nccl|gloo)")
    have_gpu = torch.cuda.is_available()
    if device == "cpu":
        if backend == "nccl":
            raise RuntimeError("--device cpu with backend rccl: RCCL needs HIP devices")
        return "gloo"
    if backend == "nccl" or device == "gpu":
        if not have_gpu:
            raise RuntimeError("a GPU run was requested (backend rccl / --device gpu) but no HIP "
                               "device is usable (torch.cuda.is_available() is False)")
        return backend or "nccl"
    if backend is not None:
        return backend
    if have_gpu:
        return "nccl"
    if _gpu_host():
        raise RuntimeError("this host exposes a GPU (/dev/kfd) but the HIP runtime is not usable; "
                           "refusing to fall back to CPU/gloo silently (pass --device cpu to "
                           "train on the CPU)")
    return "gloo"


def setup(rank: int, world_size: int, backend: str | None = None, verbose: bool = True,
          timeout_s: float | None = None, device: str | None = None) -> str:
    """Join the process group; returns the backend used (see :func:`resolve_backend`)."""
    backend = resolve_backend(backend, device)
    # a single process with no launcher-given port needs no TCP rendezvous: an in-process
    # store avoids the free-port race (a port picked here can be taken before TCPStore binds
    # it - seen as EADDRINUSE on a GPU box between back-to-back runs)
    own_store = world_size == 1 and "MASTER_PORT" not in os.environ
    ensure_master_env()
    if backend == "nccl":
        if not torch.cuda.is_available():
            raise RuntimeError("backend rccl/nccl requested but no HIP device is visible")
        torch.cuda.set_device(local_rank(rank))
    t = timeout_s or float(os.environ.get("DDP_AMD_PG_TIMEOUT", 1800))
    kw = dict(backend=backend, world_size=world_size, rank=rank,
              timeout=datetime.timedelta(seconds=t))
    if backend == "nccl":
        kw["device_id"] = torch.device("cuda", local_rank(rank))
    if own_store:
        kw["store"] = dist.HashStore()
    dist.init_process_group(**kw)
    if verbose:
        print(f"Rank: {rank} has initialized its process group with world size {world_size}",
              flush=True)
    return backend


def cleanup(verbose: bool = True):
    global _native_comm
    rank = dist.get_rank()
    _native_comm = None
    dist.destroy_process_group()
    if verbose:
        print(f"Rank {rank} cleaned up.", flush=True)


def native_comm():
    """The process-wide native RCCL communicator (created on first use, collective)."""
    global _native_comm
    if _native_comm is not None:
        return _native_comm
    from .. import native

    C = native.require()
    rank, world = dist.get_rank(), dist.get_world_size()
    store = dist.distributed_c10d._get_default_store()
    key = "ddp_amd/rccl_uid"
    if rank == 0:
        store.set(key, C.Comm.new_unique_id())
    uid = store.get(key)
    _native_comm = C.Comm(uid, rank, world, torch.cuda.current_device())
    return _native_comm
