"""Bootstrap of the direct xGMI all-reduce (csrc/runtime/xgmi.cpp, csrc/kernels/allreduce.hip).

The data plane of the fused engine's bucket all-reduces at world size > 1: one kernel per
bucket that pulls every peer's slice over its own xGMI link (two cross-GPU barriers, fixed
rank order, bitwise identical on every rank) instead of an RCCL ring - see the kernel's
header for the protocol.  SURVEY.md §5.8 (design items 3 and 4).

Bootstrap: every rank registers the flat gradient buffer and one channel per bucket,
publishes its IPC handle blob in the c10d TCPStore, maps every peer's blob, then runs a
self-test on exactly-representable patterns.  If any rank's self-test fails (or a
barrier timed out) every rank gets ``None`` back and the caller falls back to RCCL.
"""
from __future__ import annotations

import itertools
import sys

import torch
import torch.distributed as dist

from .. import native

_gen = itertools.count()


def _pattern(n: int, rank: int, device) -> torch.Tensor:
    i = torch.arange(n, device=device, dtype=torch.int64)
    return (((i * 7 + rank * 13) % 101).to(torch.float32) * 0.25 - 12.0)


def create_xgmi(grads: torch.Tensor, buckets, rank: int, world: int, store=None,
                self_test: bool = True, verbose: bool = True):
    """XgmiComm over ``grads`` (flat fp32, CUDA) with one channel per ``(offset, numel)``
    bucket, or ``None`` when the direct path is unusable here (collective: every rank
    must call it with the same buckets)."""
    C = native.require()
    store = store or dist.distributed_c10d._get_default_store()
    gen = next(_gen)
    key = f"ddp_amd/xgmi/{gen}"
    ok = True
    x = None
    try:
        x = C.XgmiComm(rank, world, grads.device.index)
        for off, n in buckets:
            x.add_channel(int(off), int(n))
        x.set_data(grads)
        store.set(f"{key}/h/{rank}", x.export_handles())
        blobs = [store.get(f"{key}/h/{r}") for r in range(world)]
        x.import_handles(blobs)
    except Exception as e:  # noqa: BLE001 - report, agree, fall back
        if verbose:
            print(f"[ddp_amd] rank {rank}: xGMI setup failed ({e}); using RCCL", file=sys.stderr)
        ok = False
    if ok and self_test:
        ok = _self_test(x, grads, buckets, rank, world)
    store.set(f"{key}/ok/{rank}", b"1" if ok else b"0")
    agreed = all(store.get(f"{key}/ok/{r}") == b"1" for r in range(world))
    if not agreed:
        if verbose and ok:
            print(f"[ddp_amd] rank {rank}: a peer's xGMI self-test failed; using RCCL", file=sys.stderr)
        return None
    return x


def _self_test(x, grads, buckets, rank, world) -> bool:
    saved = grads.detach().clone()
    try:
        stream = torch.cuda.current_stream()
        for rounds in range(3):  # exercises both stage-buffer parities
            for ch, (off, n) in enumerate(buckets):
                grads[off:off + n].copy_(_pattern(n, rank + rounds, grads.device))
            stream.synchronize()
            for ch in range(len(buckets)):
                x.all_reduce(ch)
            stream.synchronize()
            if x.error_flags():
                print(f"[ddp_amd] rank {rank}: xGMI barrier timeout in self-test", file=sys.stderr)
                return False
            for off, n in buckets:
                want = sum(_pattern(n, r + rounds, grads.device) for r in range(world))
                if not torch.equal(grads[off:off + n], want):
                    print(f"[ddp_amd] rank {rank}: xGMI self-test mismatch", file=sys.stderr)
                    return False
        return True
    finally:
        grads.copy_(saved)
        torch.cuda.current_stream().synchronize()


def pick_data_plane(x, comm, grads: torch.Tensor, buckets, rank: int, iters: int = 30, store=None):
    """Time the engine's two bucket all-reduces over the xGMI kernel and over RCCL on
    this node (``iters`` back-to-back pairs each, after a warm-up); returns
    ``(use_xgmi, {"xgmi": us, "rccl": us})`` with rank 0's measurement and decision
    broadcast through the store, so every rank picks the same data plane.  The
    gradient buffer's contents are clobbered (the engine rewrites every bucket each step)."""
    store = store or dist.distributed_c10d._get_default_store()
    gen = next(_gen)
    views = [grads[off:off + n] for off, n in buckets]

    def t_xgmi():
        for ch in range(len(buckets)):
            x.all_reduce(ch)

    def t_rccl():
        for v in views:
            comm.all_reduce(v)

    def timed(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1000.0 / iters

    tx = timed(t_xgmi)
    tr = timed(t_rccl)
    ok = x.error_flags() == 0
    key = f"ddp_amd/xgmi/pick/{gen}"
    if rank == 0:
        store.set(key, f"{int(ok and tx <= tr)} {tx:.2f} {tr:.2f}".encode())
    use, a, b = store.get(key).decode().split()
    return use == "1", {"xgmi": float(a), "rccl": float(b)}
