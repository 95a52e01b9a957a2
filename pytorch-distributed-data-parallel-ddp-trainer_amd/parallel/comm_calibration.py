"""Calibration of the xGMI all-reduce cost model.

``bucket_model.XgmiCost`` prices a bucket all-reduce as

    t = launch_us + barriers * barrier_us + link_bytes / (link_gbps * link_eff)

(two-shot: 2 barriers, 2 x bytes / N per link; one-shot: 1 barrier, the whole bucket per
link).  Its three free constants were guesses in round 3.  This module measures them:

* :func:`sweep_xgmi` times the real bucket kernels (kernels/allreduce.hip, both kinds) over
  a range of bucket sizes on the job's own ranks - collective, a few milliseconds;
* :func:`fit_cost` least-squares fits ``launch_us``, ``barrier_us`` and the link rate to those
  samples (all three enter linearly: t = a + b * barriers + c * link_bytes);
* :func:`save` / :func:`load` keep fits with their provenance (world size, topology - "xgmi"
  when every rank has its own GPU, "same-gpu" for the one-GPU rehearsals -, device, date)
  in ``xgmi_calibration.json`` next to this file.

``XgmiCost.calibrated(world)`` uses a stored fit of the SAME world size measured on real
peers ("xgmi"); same-GPU fits are kept as a record only (their "links" are one GPU's own
memory).  ``bench.py`` at N > 1 sweeps and fits BEFORE it builds the engine (untimed),
plans the buckets with that fit (``XgmiCost.from_fit``: ``config.bucket_plan`` records
``cost_source = "fit:<topology>"``), reports it (``config.comm_calibration``) and, on real
xGMI peers, stores it under ``xgmi/<N>`` with its provenance for later runs.
"""
from __future__ import annotations

import datetime
import json
import os

import torch

CAL_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "xgmi_calibration.json")
SWEEP_ELEMS = (1024, 8192, 32768, 131072, 262144, 524288, 1048576)


def link_bytes(kind: str, nbytes: float, world: int) -> float:
    return nbytes if kind == "oneshot" else 2.0 * nbytes / world


def barriers(kind: str) -> int:
    return 1 if kind == "oneshot" else 2


def fit_cost(samples, world: int, link_gbps: float = 153.0) -> dict:
    """Least-squares fit of (launch_us, barrier_us, link_eff) to [(nbytes, kind, us), ...].

    Needs both kernel kinds (one-shot and two-shot) so the barrier term is separable from the
    fixed term.  Negative fits are clamped to 0 (and the rest refitted)."""
    import numpy as np

    kinds = {k for _, k, _ in samples}
    if kinds != {"oneshot", "twoshot"}:
        raise ValueError("fit_cost needs one-shot and two-shot samples")
    A = np.array([[1.0, barriers(k), link_bytes(k, b, world)] for b, k, _ in samples])
    y = np.array([t for _, _, t in samples])
    free = [0, 1, 2]
    x = np.zeros(3)
    for _ in range(3):  # non-negativity by elimination (tiny problem)
        sol, *_ = np.linalg.lstsq(A[:, free], y, rcond=None)
        x[:] = 0.0
        x[free] = sol
        neg = [i for i in free if x[i] < 0]
        if not neg:
            break
        free = [i for i in free if i not in neg]
        x[neg] = 0.0
    pred = A @ x
    inv_rate = x[2]  # us per byte
    eff = (1.0 / (inv_rate * link_gbps * 1e3)) if inv_rate > 0 else 1.0
    return {"launch_us": float(x[0]), "barrier_us": float(x[1]), "link_eff": float(eff),
            "link_gbps": link_gbps, "rms_us": float(np.sqrt(np.mean((pred - y) ** 2))), "n": len(samples)}


def sweep_xgmi(rank: int, world: int, device, elems=SWEEP_ELEMS, iters: int = 20, store=None) -> list:
    """Time the two-shot and one-shot bucket kernels on every size (collective).  Returns
    [(nbytes, kind, us)]; [] when the direct path is unusable here."""
    from .xgmi import create_xgmi

    n_max = max(elems)
    buf = torch.zeros(n_max, device=device)
    buckets = [(0, int(n)) for n in elems]
    x = create_xgmi(buf, buckets, rank, world, store=store, oneshot=tuple(range(len(buckets))), verbose=False)
    if x is None:
        return []
    out = []
    nb = len(buckets)
    for b, n in enumerate(elems):
        for kind, ch in (("twoshot", b), ("oneshot", nb + b)):
            for _ in range(3):
                x.all_reduce(ch)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(iters):
                x.all_reduce(ch)
            e1.record()
            e1.synchronize()
            out.append((4 * int(n), kind, e0.elapsed_time(e1) * 1000.0 / iters))
    bad = x.error_flags() != 0
    # every rank finished its kernels before any rank drops its channels (the peers' last
    # all-gathers read this rank's stage buffers)
    torch.cuda.synchronize()
    if store is not None or world > 1:
        import torch.distributed as dist

        st = store or dist.distributed_c10d._get_default_store()
        key = f"ddp_amd/cal_sweep_done/{next(_sweep_gen)}"
        st.set(f"{key}/{rank}", b"1")
        for r in range(world):
            st.get(f"{key}/{r}")
    del x
    return [] if bad else out


_sweep_gen = iter(range(1 << 30))


def topology(world: int, store=None, rank: int = 0) -> str:
    """"xgmi" when every rank has a GPU of its own, else "same-gpu" (rehearsal)."""
    if world <= 1:
        return "single"
    from .. import native
    from .xgmi import max_sharing

    import torch.distributed as dist

    store = store or dist.distributed_c10d._get_default_store()
    key = "ddp_amd/cal_topo"
    store.set(f"{key}/{rank}", native.require().pci_bus_id(torch.cuda.current_device()).encode())
    return "xgmi" if max_sharing(store.get(f"{key}/{r}").decode() for r in range(world)) == 1 else "same-gpu"


def load(path: str = CAL_PATH) -> dict:
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return {}


def save(fit: dict, world: int, topo: str, path: str = CAL_PATH, extra: dict | None = None) -> dict:
    """Store a fit under key ``"<topo>/<world>"`` with its provenance; returns the record."""
    rec = dict(fit)
    rec.update({"world": world, "topology": topo,
                "device": torch.cuda.get_device_name() if torch.cuda.is_available() else None,
                "date": datetime.date.today().isoformat()})
    if extra:
        rec.update(extra)
    allc = load(path)
    allc[f"{topo}/{world}"] = rec
    with open(path, "w") as f:
        json.dump(allc, f, indent=1, sort_keys=True)
    return rec


def calibrate(rank: int, world: int, device, store=None) -> dict | None:
    """Sweep + fit on rank 0's samples, shared through the store so every rank gets the same
    constants (collective).  None when the direct path is unusable."""
    import torch.distributed as dist

    store = store or dist.distributed_c10d._get_default_store()
    samples = sweep_xgmi(rank, world, device, store=store)
    key = "ddp_amd/cal_fit"
    if rank == 0:
        fit = fit_cost(samples, world) if samples else None
        if fit is not None:
            fit["samples"] = [[b, k, round(t, 3)] for b, k, t in samples]
        store.set(key, json.dumps(fit).encode())
    return json.loads(store.get(key).decode())
