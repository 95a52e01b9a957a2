"""Bootstrap of the direct xGMI all-reduce (csrc/runtime/xgmi.cpp, csrc/kernels/allreduce.hip).

The data plane of the fused engine's bucket all-reduces at world size > 1.  Each bucket
gets one kernel that pulls over the xGMI links directly instead of running an RCCL ring:

* two-shot: every rank pulls its own slice of the bucket from every peer over that peer's
  link, sums in fixed rank order, then gathers the reduced slices back (two cross-GPU
  barriers, bitwise identical on every rank);
* one-shot (small buckets): every rank pulls every peer's whole bucket and sums it
  itself (one barrier).

See the kernel's header for the protocol.  SURVEY.md §5.8 (design items 3 and 4), §7.3
step 7.

Bootstrap:

1. Every rank registers the flat gradient buffer and one channel per (bucket, mode).
2. It publishes its IPC handle blob in the c10d TCPStore and maps every peer's blob.
3. It runs a self-test on exactly-representable patterns on every channel.

If any rank's self-test fails (or a barrier timed out), every rank gets ``None`` back and
the caller falls back to RCCL.  :func:`pick_data_plane` then times the candidate plans on
the node and keeps the fastest.
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


# Grid of one bucket kernel.  The kernel spins in its cross-GPU barriers with one block
# per CU it occupies, and a spinning block pins registers a full-width compute block would
# need: an all-reduce that overlaps the backward (the module reducer) keeps a small grid
# (MODULE_GRID_CAP: 2 x 16 B quads x 8 ranks per lane still keep ~2 MB in flight), one
# that runs alone (the fused engine's, after the conv backward) may take the whole chip.
ENGINE_GRID_CAP = 256
MODULE_GRID_CAP = 32
# Ranks sharing one GPU (same-GPU rehearsals): every rank's spinning grid must leave room
# for the others' compute kernels, or a rank that has not reached the all-reduce yet can
# never get its producers onto a CU (a cross-process deadlock until the barrier timeout).
SHARED_GPU_CUS = 64


def grid_cap_for(requested: int, ranks_on_device: int) -> int:
    """Blocks per bucket kernel for ``requested`` and the number of ranks on the most
    shared GPU of the job (every rank must pass the same value: see :func:`max_sharing`)."""
    if ranks_on_device > 1:
        return max(4, min(requested, SHARED_GPU_CUS // ranks_on_device))
    return requested


def max_sharing(bus_ids) -> int:
    """Ranks on the most shared device, from every rank's PCI bus id.

    The bucket kernel's barriers pair block b of one rank with block b of each peer, and
    its publish / reduce passes assume one thread-to-quad map on every rank, so every rank
    must size its grid from the SAME number - the job-wide maximum, not its own device's
    count (3 ranks on 2 GPUs: ranks 0 and 2 share one, rank 1 is alone; all three use 2)."""
    counts: dict = {}
    for b in bus_ids:
        counts[b] = counts.get(b, 0) + 1
    return max(counts.values()) if counts else 1


def check_blocks_agree(blocks_per_rank) -> None:
    """Raise unless every rank built every channel with the same grid (list per rank)."""
    first = list(blocks_per_rank[0])
    for r, b in enumerate(blocks_per_rank):
        if list(b) != first:
            raise RuntimeError(f"xGMI channel grids differ across ranks (rank 0 {first}, rank {r} {list(b)})")


def create_xgmi(grads: torch.Tensor, buckets, rank: int, world: int, store=None,
                self_test: bool = True, verbose: bool = True, oneshot=(), grid_cap: int = ENGINE_GRID_CAP):
    """Build an XgmiComm over ``grads`` (flat fp32, CUDA), or return ``None`` when the direct
    path is unusable here.

    Channels: ``0..len(buckets)-1`` are two-shot channels, one per ``(offset, numel)``
    bucket. They are followed by one one-shot channel per bucket index listed in
    ``oneshot`` (:func:`channel_plan` maps buckets to channels).

    Collective: every rank must call it with the same buckets."""
    C = native.require()
    store = store or dist.distributed_c10d._get_default_store()
    gen = next(_gen)
    key = f"ddp_amd/xgmi/{gen}"
    chans = [(int(o), int(n), False) for o, n in buckets] + \
            [(int(buckets[b][0]), int(buckets[b][1]), True) for b in oneshot]
    ok = True
    x = None
    try:
        x = C.XgmiComm(rank, world, grads.device.index)
        bus = x.bus_id()
        store.set(f"{key}/bus/{rank}", bus.encode())
        cap = grid_cap_for(grid_cap, max_sharing(store.get(f"{key}/bus/{r}").decode() for r in range(world)))
        for off, n, one in chans:
            x.add_channel(off, n, one, cap)
        mine = [x.blocks(ch) for ch in range(len(chans))]
        store.set(f"{key}/blk/{rank}", ",".join(map(str, mine)).encode())
        check_blocks_agree([[int(v) for v in store.get(f"{key}/blk/{r}").decode().split(",") if v]
                            for r in range(world)])
        x.set_data(grads)
        store.set(f"{key}/h/{rank}", x.export_handles())
        blobs = [store.get(f"{key}/h/{r}") for r in range(world)]
        x.import_handles(blobs)
    except Exception as e:  # noqa: BLE001 - report, agree, fall back
        if verbose:
            print(f"[ddp_amd] rank {rank}: xGMI setup failed ({e}); using RCCL", file=sys.stderr)
        ok = False
    if ok and self_test:
        ok = _self_test(x, grads, chans, rank, world)
    store.set(f"{key}/ok/{rank}", b"1" if ok else b"0")
    agreed = all(store.get(f"{key}/ok/{r}") == b"1" for r in range(world))
    if not agreed:
        if verbose and ok:
            print(f"[ddp_amd] rank {rank}: a peer's xGMI self-test failed; using RCCL", file=sys.stderr)
        return None
    return x


_PHASES = {0: "B0 (entry: gradients final)", 1: "B1 (reduce-scatter done)", 2: "one-shot publish"}


def describe_xgmi_error(code: int) -> str:
    """Readable form of an XgmiComm error word (launchers.h ``xgmi_error_code``): which
    block of this rank waited for which peer at which barrier until the spin bound."""
    code = int(code)
    if code == 0:
        return "ok"
    if code & 0x80000000:
        blk, peer, phase = (code >> 12) & 0x7FFFF, (code >> 4) & 0xFF, code & 0xF
        return (f"block {blk} timed out waiting for peer rank {peer} at barrier "
                f"{_PHASES.get(phase, phase)}")
    return f"error word {code:#x}"


def channel_plan(nbuckets: int, oneshot=()) -> dict:
    """``{(bucket, oneshot): channel}`` for a comm built by ``create_xgmi(..., oneshot=...)``."""
    plan = {(b, False): b for b in range(nbuckets)}
    for k, b in enumerate(oneshot):
        plan[(b, True)] = nbuckets + k
    return plan


def _self_test(x, grads, chans, rank, world) -> bool:
    saved = grads.detach().clone()
    try:
        stream = torch.cuda.current_stream()
        for ch, (off, n, _) in enumerate(chans):
            for rounds in range(3):  # exercises both stage-buffer parities
                grads[off:off + n].copy_(_pattern(n, rank + rounds, grads.device))
                stream.synchronize()
                x.all_reduce(ch)
                stream.synchronize()
                if x.error_flags():
                    print(f"[ddp_amd] rank {rank}: xGMI self-test: {describe_xgmi_error(x.error_flags())}",
                          file=sys.stderr)
                    return False
                want = sum(_pattern(n, r + rounds, grads.device) for r in range(world))
                if not torch.equal(grads[off:off + n], want):
                    print(f"[ddp_amd] rank {rank}: xGMI self-test mismatch (channel {ch})", file=sys.stderr)
                    return False
        return True
    finally:
        grads.copy_(saved)
        torch.cuda.current_stream().synchronize()


# RCCL algorithm / protocol candidates of ``--comm tune``: RCCL reads
# NCCL_ALGO / NCCL_PROTO when it tunes a NEW communicator, so each candidate is a fresh
# communicator created with them set.
RCCL_CANDIDATES = (("Ring", "Simple"), ("Ring", "LL"), ("Ring", "LL128"), ("Tree", "Simple"), ("Tree", "LL"))


def rccl_candidate_comms(rank: int, world: int, store=None, candidates=RCCL_CANDIDATES) -> dict:
    """{"rccl:<algo>/<proto>": communicator} for every candidate whose communicator
    initialised on EVERY rank (collective; a candidate that failed anywhere is left out)."""
    import os

    from ..engine.fused_step import agree

    C = native.require()
    store = store or dist.distributed_c10d._get_default_store()
    gen = next(_gen)
    out = {}
    for i, (algo, proto) in enumerate(candidates):
        key = f"ddp_amd/rccl_cand/{gen}/{i}"
        saved = {k: os.environ.get(k) for k in ("NCCL_ALGO", "NCCL_PROTO")}
        os.environ["NCCL_ALGO"], os.environ["NCCL_PROTO"] = algo, proto
        comm = None
        # vote BEFORE the collective init: a rank that cannot even start this
        # candidate must not leave the others blocked inside ncclCommInitRank
        uid = b""
        try:
            if rank == 0:
                try:
                    uid = C.Comm.new_unique_id()
                finally:
                    store.set(key, uid)
            uid = store.get(key)
        except Exception as e:  # noqa: BLE001
            print(f"[ddp_amd] rank {rank}: RCCL {algo}/{proto} id exchange failed ({e})", file=sys.stderr)
            uid = b""
        if not agree(store, key + "/ready", rank, world, len(uid) > 0):
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
            continue
        try:
            comm = C.Comm(uid, rank, world, torch.cuda.current_device())
        except Exception as e:  # noqa: BLE001 - an unsupported combination on this node
            print(f"[ddp_amd] rank {rank}: RCCL {algo}/{proto} communicator failed ({e})", file=sys.stderr)
            comm = None
        finally:
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        if agree(store, key + "/ok", rank, world, comm is not None):
            out[f"rccl:{algo}/{proto}"] = comm
    return out


def pick_data_plane(x, comm, grads: torch.Tensor, buckets, rank: int, iters: int = 30, store=None,
                    oneshot=(), rccl_variants: dict | None = None):
    """Time the engine's bucket all-reduces under every available plan on this node.

    Candidates:

    * ``"xgmi"``: two-shot kernels for every bucket;
    * ``"xgmi1"``: the same, except the one-shot kernel for the buckets in ``oneshot``;
    * ``"rccl"``: RCCL (the default communicator);
    * ``"rccl:<algo>/<proto>"``: one per communicator in ``rccl_variants``
      (:func:`rccl_candidate_comms`) - timed only because it initialised everywhere.

    Each candidate runs ``iters`` back-to-back rounds after a warm-up.  Returns
    ``(plan, {plan: us}, comm)``: ``plan`` is the fastest candidate by rank 0's measurement,
    broadcast through the store so that every rank picks the same one; ``comm`` the RCCL
    communicator to use when the plan is an RCCL one.

    The gradient buffer's contents are clobbered; the engine rewrites every bucket each
    step."""
    store = store or dist.distributed_c10d._get_default_store()
    gen = next(_gen)
    nb = len(buckets)
    chans = channel_plan(nb, oneshot)
    views = [grads[off:off + n] for off, n in buckets]
    plans = {"xgmi": [chans[(b, False)] for b in range(nb)]}
    if oneshot:
        plans["xgmi1"] = [chans[(b, b in oneshot)] for b in range(nb)]

    def run_x(chs):
        def f():
            for ch in chs:
                x.all_reduce(ch)
        return f

    def run_rccl(c):
        def f():
            for v in views:
                c.all_reduce(v)
        return f

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

    times = {name: timed(run_x(chs)) for name, chs in plans.items()}
    comms = {}
    if comm is not None:
        comms["rccl"] = comm
    comms.update(rccl_variants or {})
    for name, c in comms.items():
        times[name] = timed(run_rccl(c))
    ok = x.error_flags() == 0
    key = f"ddp_amd/xgmi/pick/{gen}"
    if rank == 0:
        cand = {k: v for k, v in times.items() if ok or k.startswith("rccl")}
        best = min(cand, key=cand.get)
        store.set(key, (best + " " + " ".join(f"{k}={v:.2f}" for k, v in times.items())).encode())
    parts = store.get(key).decode().split()
    best = parts[0]
    measured = {k: float(v) for k, v in (p.split("=") for p in parts[1:])}
    return best, measured, comms.get(best)
