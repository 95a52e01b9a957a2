"""Gradient-bucket plan from a cost model of the direct xGMI all-reduce.

The reference inherits torch DDP's size rule - first bucket 1 MiB, then 25 MiB
(/root/reference/train_ddp.py:34, torch/nn/parallel/distributed.py:1204-1245) - a rule
tuned for NCCL rings over NVLink/IB.  On an 8x MI355X node every GPU has 7 point-to-point
xGMI links (~153 GB/s each way) and our bucket all-reduce is ONE kernel
(kernels/allreduce.hip):

* two-shot: entry barrier, reduce-scatter (each rank pulls its 1/N slice from the N-1
  peers over N-1 links at once), barrier, all-gather -> 2 barriers + 2 x bytes/N per link;
* one-shot: every rank pulls the whole bucket from every peer -> 1 barrier + bytes per link.

So a bucket costs  t(b) = launch + barriers(kind) * barrier + link_bytes(kind, b) / link_rate,
and the comm stream runs the buckets one after another, each no earlier than its last
gradient is final.  With the time at which every gradient becomes final (a per-layer
backward-time estimate, or the fused engine's two stages), :func:`plan_buckets` picks
the contiguous grouping (in gradient-ready order) that minimises the completion time of
the LAST all-reduce - the only comm time left on the critical path - by dynamic
programming; ties go to fewer buckets.  Each bucket also gets its kernel (one-shot below
the crossover size, :meth:`XgmiCost.oneshot_max_elems`).

The fixed terms are defaults until measured: ``barrier_us`` is a cross-GPU flag round trip
(a system-scope store seen by a peer's poll over xGMI, ~1.5 us each way), ``launch_us`` the
graph-node/event hop of one more bucket kernel on the comm stream, ``link_eff`` the share
of a link's 153 GB/s the pulls reach.  ``parallel/comm_calibration.py`` fits all three to
timed sweeps of the real kernels; :meth:`XgmiCost.calibrated` uses a stored fit measured on
real peers at the same world size (``xgmi_calibration.json``, with provenance), and
``bench.py`` refits on every N > 1 run (``config.comm_calibration``).
"""
from __future__ import annotations

import dataclasses

import torch
import torch.nn as nn


# Largest bucket (fp32 elements) a one-shot channel can take: the whole bucket must fit one
# kernel grid (1024 x 256, kernels/launchers.h XGMI_MAX_BLOCKS x XGMI_THREADS) - larger
# buckets always run two-shot, whatever the model's crossover says.  The engine (fused_step.py), the
# module path (ddp.py), the planner and describe() all apply it, so a plan is priced with
# the kernel that will actually run it.
ONESHOT_MAX_ELEMS = 1024 * 256


@dataclasses.dataclass
class XgmiCost:
    world: int
    link_gbps: float = 153.0  # one xGMI link, one direction
    link_eff: float = 0.7     # achievable share with system-scope 4-byte pulls
    barrier_us: float = 3.0   # one cross-GPU barrier
    launch_us: float = 1.5    # one more bucket kernel on the comm stream (graph node + event)
    # where the constants came from: "default" (guesses), "stored:<key>" (a fit measured on
    # real peers earlier, xgmi_calibration.json) or "fit:<topology>" (measured by this job,
    # before its engine was built - bench.py at N > 1)
    source: str = dataclasses.field(default="default", compare=False)

    @classmethod
    def calibrated(cls, world: int, path: str | None = None) -> "XgmiCost":
        """The model with the constants of a stored fit for this world size measured on real
        xGMI peers (comm_calibration.json key "xgmi/<world>"), else the defaults."""
        from .comm_calibration import CAL_PATH, load

        rec = load(path or CAL_PATH).get(f"xgmi/{world}")
        if not rec:
            return cls(world)
        return cls.from_fit(world, rec, source=f"stored:xgmi/{world}")

    @classmethod
    def from_fit(cls, world: int, fit: dict, source: str = "fit") -> "XgmiCost":
        """The model with a fit's constants (comm_calibration.fit_cost / calibrate)."""
        return cls(world, link_gbps=fit.get("link_gbps", 153.0), link_eff=fit["link_eff"],
                   barrier_us=fit["barrier_us"], launch_us=fit["launch_us"], source=source)

    def _link_us(self, nbytes: float) -> float:
        return nbytes / (self.link_gbps * self.link_eff * 1e3)  # bytes / (GB/s) -> us

    def two_shot_us(self, nbytes: float) -> float:
        if self.world <= 1:
            return self.launch_us
        return self.launch_us + 2 * self.barrier_us + 2 * self._link_us(nbytes / self.world)

    def one_shot_us(self, nbytes: float) -> float:
        if self.world <= 1:
            return self.launch_us
        return self.launch_us + self.barrier_us + self._link_us(nbytes)

    def allreduce(self, nbytes: float) -> tuple[float, str]:
        """(predicted us, kernel) of one bucket all-reduce - the kernel the engine runs for it:
        one-shot only up to :meth:`oneshot_cap_elems`."""
        b = self.two_shot_us(nbytes)
        if nbytes / 4 > self.oneshot_cap_elems():
            return b, "twoshot"
        a = self.one_shot_us(nbytes)
        return (a, "oneshot") if a <= b else (b, "twoshot")

    def oneshot_cap_elems(self) -> int:
        """Largest bucket that gets a one-shot channel: the model's crossover, capped by the
        kernel's grid limit (ONESHOT_MAX_ELEMS)."""
        return min(ONESHOT_MAX_ELEMS, self.oneshot_max_elems())

    def oneshot_max_elems(self) -> int:
        """Largest fp32 bucket for which the one-shot kernel is predicted faster: one barrier
        saved against (N - 2) / N of the bucket's bytes more per link.
        ``DDP_AMD_XGMI_ONESHOT_MAX`` overrides it (sweeps, A/B)."""
        import os

        if os.environ.get("DDP_AMD_XGMI_ONESHOT_MAX"):
            return int(os.environ["DDP_AMD_XGMI_ONESHOT_MAX"])
        if self.world <= 2:
            return 1 << 30  # N <= 2: one-shot moves no more bytes per link than two-shot
        per_byte = self._link_us(1.0) * (1.0 - 2.0 / self.world)
        return int(self.barrier_us / per_byte / 4)


def plan_buckets(sizes: list[int], ready_us: list[float], cost: XgmiCost, max_buckets: int = 16):
    """Optimal contiguous bucketing of gradients in ready order.

    ``sizes[i]``: bytes of gradient i; ``ready_us[i]``: when it is final (non-decreasing).
    Returns ``(bounds, finish_us)`` with ``bounds`` = [(start, end), ...] index ranges and
    the predicted completion time of the last all-reduce."""
    n = len(sizes)
    if n == 0:
        return [], 0.0
    if any(ready_us[i] > ready_us[i + 1] + 1e-9 for i in range(n - 1)):
        raise ValueError("ready times must be non-decreasing in gradient-ready order")
    pre = [0]
    for s in sizes:
        pre.append(pre[-1] + s)
    INF = float("inf")
    # best[k][j]: earliest finish of the k-th bucket ending at j (first j gradients in k buckets)
    best = [[INF] * (n + 1) for _ in range(max_buckets + 1)]
    arg = [[-1] * (n + 1) for _ in range(max_buckets + 1)]
    best[0][0] = 0.0
    for k in range(1, max_buckets + 1):
        for j in range(1, n + 1):
            for i in range(k - 1, j):
                if best[k - 1][i] == INF:
                    continue
                t = max(ready_us[j - 1], best[k - 1][i]) + cost.allreduce(pre[j] - pre[i])[0]
                if t < best[k][j] - 1e-9:
                    best[k][j], arg[k][j] = t, i
    # fewest buckets within 0.5 % of the best finish time
    top = min(best[k][n] for k in range(1, max_buckets + 1))
    k = next(k for k in range(1, max_buckets + 1) if best[k][n] <= top * 1.005 + 1e-9)
    top = best[k][n]
    bounds, j = [], n
    while k > 0:
        i = arg[k][j]
        bounds.append((i, j))
        j, k = i, k - 1
    return bounds[::-1], top


# ---------------------------------------------------------------- gradient-ready times
def backward_times_us(model: nn.Module, sample: torch.Tensor, tflops: float = 160.0,
                      hbm_tbps: float = 4.0) -> dict:
    """Estimated backward time (us) of every leaf module with parameters, from ONE forward
    of ``sample`` (its batch is the per-rank batch): convolutions / linears cost 2x their
    forward FLOPs (data + weight gradient) at ``tflops``, BatchNorm three passes over its
    bf16 activation at ``hbm_tbps`` (the step's measured rates: ResNet-18 runs ~156 TFLOP/s -
    348 GFLOP per B = 32 step in 2.23 ms, profiles/r2_final).
    Keys are module names."""
    est, hooks = {}, []

    def hook(name):
        # by weight shape, so the package's own layer classes count too: 4-d = convolution
        # ([co][ci/groups][kh][kw] or OHWI - the product of the last three is the MACs per
        # output either way), 2-d = linear, 1-d with running stats = BatchNorm
        def f(m, inp, out):
            w = getattr(m, "weight", None)
            o = out.numel() if torch.is_tensor(out) else 0
            if w is not None and w.dim() == 4:
                est[name] = 2 * (2.0 * o * w[0].numel()) / (tflops * 1e6)
            elif w is not None and w.dim() == 2:
                est[name] = 2 * (2.0 * o * w.shape[1]) / (tflops * 1e6)
            elif getattr(m, "running_mean", None) is not None:
                est[name] = 3 * 2.0 * o / (hbm_tbps * 1e6)
            else:
                est[name] = 0.0
        return f

    patched = []
    for name, m in model.named_modules():
        if any(True for _ in m.parameters(recurse=False)):
            hooks.append(m.register_forward_hook(hook(name)))
            fn = getattr(m, "forward_nchw", None)  # layers.Conv2d: called directly, not through __call__
            if fn is not None:
                def wrapped(*a, _fn=fn, _m=m, _h=hook(name), **k):
                    out = _fn(*a, **k)
                    _h(_m, a, out)
                    return out
                m.forward_nchw = wrapped
                patched.append(m)
    try:
        with torch.no_grad():
            model(sample)
    finally:
        for h in hooks:
            h.remove()
        for m in patched:
            del m.forward_nchw  # back to the class method
    return est


def ready_times_us(names: list[str], module_of: dict, bwd_us: dict) -> list[float]:
    """Time each gradient (``names`` in gradient-ready order) becomes final: the backward
    runs the modules in that order, a module's gradients are final when it is done."""
    t, seen, out = 0.0, set(), []
    for n in names:
        mod = module_of[n]
        if mod not in seen:
            seen.add(mod)
            t += bwd_us.get(mod, 0.0)
        out.append(t)
    return out


def module_plan(fs, model: nn.Module, sample: torch.Tensor, world: int, cost: XgmiCost | None = None):
    """Bucket plan (lists of parameter names, gradient-ready order) for the module path."""
    cost = cost or XgmiCost(world)
    module_of = {n: n.rsplit(".", 1)[0] if "." in n else "" for n in fs.names}
    sizes = [fs.numels[n] * 4 for n in fs.names]
    ready = ready_times_us(fs.names, module_of, backward_times_us(model, sample))
    bounds, finish = plan_buckets(sizes, ready, cost)
    return [fs.names[i:j] for i, j in bounds], finish


def engine_plan(fs, world: int, cost: XgmiCost | None = None, fc_ready_us: float = 2.0,
                conv_ready_us: float = 18.0):
    """Bucket plan of the fused SimpleCNN engine: the fc gradients are all final when the fc
    weight-gradient kernel ends (stage 0), the conv gradients when the conv backward's
    fused reduction ends (stage 1) - within a stage everything is final at once."""
    cost = cost or XgmiCost(world)
    sizes = [fs.numels[n] * 4 for n in fs.names]
    ready = [fc_ready_us if n.startswith("fl.") else conv_ready_us for n in fs.names]
    bounds, finish = plan_buckets(sizes, ready, cost)
    return [fs.names[i:j] for i, j in bounds], finish


def describe(buckets, fs, cost: XgmiCost, ranges=None) -> list[dict]:
    """Per-bucket record for logs / bench config: size, the kernel that runs it (one-shot
    only within :meth:`XgmiCost.oneshot_cap_elems`, as the engine decides - by the bucket's
    range in the flat buffer when ``ranges`` is given), predicted us, and where the cost
    constants came from."""
    out = []
    cap = cost.oneshot_cap_elems()
    for i, b in enumerate(buckets):
        nbytes = sum(fs.numels[n] * 4 for n in b)
        n_elems = ranges[i][1] if ranges is not None else nbytes // 4
        kind = "oneshot" if n_elems <= cap else "twoshot"
        us = cost.one_shot_us(nbytes) if kind == "oneshot" else cost.two_shot_us(nbytes)
        out.append({"params": len(b), "bytes": nbytes, "elems": int(n_elems), "kernel": kind,
                    "pred_us": round(us, 2), "cost_source": cost.source})
    return out
