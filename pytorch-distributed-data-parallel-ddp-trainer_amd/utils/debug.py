"""Collective-sequence fingerprinting.

The reference's resume path issues a *different* collective sequence on rank 0
than on the other ranks (bug B7: rank 0 broadcasts 30 more times), which hangs
or corrupts state.  :class:`CollectiveTracer` records every c10d collective a
rank issues - op name, dtype, shape, src/dst - and :meth:`verify` all-gathers a
hash of the sequence so that divergence raises an error naming the first
mismatching call, instead of deadlocking.

Enabled process-wide with ``DDP_AMD_DEBUG=1`` (``maybe_enable()``) or used as a
context manager in tests::

    with CollectiveTracer() as tr:
        ...collectives...
        tr.verify()
"""
from __future__ import annotations

import functools
import hashlib
import os

import torch
import torch.distributed as dist

_OPS = ("broadcast", "all_reduce", "all_gather", "all_gather_into_tensor", "reduce_scatter",
        "reduce_scatter_tensor", "barrier", "reduce", "scatter", "gather", "all_to_all_single",
        "broadcast_object_list", "all_gather_object")


class CollectiveDivergence(RuntimeError):
    pass


class CollectiveTracer:
    def __init__(self):
        self.log: list[tuple] = []
        self._orig = {}
        self._inside = 0

    def _wrap(self, name, fn):
        @functools.wraps(fn)
        def w(*args, **kwargs):
            if self._inside == 0:  # only the outermost call (object collectives nest)
                shape = None
                t = args[0] if args else kwargs.get("tensor")
                if torch.is_tensor(t):
                    shape = (str(t.dtype), tuple(t.shape))
                elif isinstance(t, list):
                    shape = ("list", len(t))
                root = kwargs.get("src", kwargs.get("dst", args[1] if len(args) > 1 and isinstance(args[1], int) else None))
                self.log.append((name, shape, root))
            self._inside += 1
            try:
                return fn(*args, **kwargs)
            finally:
                self._inside -= 1
        return w

    def __enter__(self):
        for op in _OPS:
            fn = getattr(dist, op, None)
            if fn is not None:
                self._orig[op] = fn
                setattr(dist, op, self._wrap(op, fn))
        return self

    def __exit__(self, *exc):
        for op, fn in self._orig.items():
            setattr(dist, op, fn)
        self._orig.clear()
        return False

    def fingerprint(self) -> str:
        return hashlib.sha256(repr(self.log).encode()).hexdigest()[:16]

    def verify(self, group=None):
        """Collective itself: every rank must call it at the same point."""
        saved = dict(self._orig)
        self.__exit__(None, None, None)  # do not trace the check itself
        try:
            mine = (self.fingerprint(), len(self.log), self.log)
            allv = [None] * dist.get_world_size(group)
            dist.all_gather_object(allv, mine, group=group)
        finally:
            if saved:
                self.__enter__()
        ref = allv[0]
        for r, v in enumerate(allv):
            if v[0] != ref[0]:
                n = min(len(v[2]), len(ref[2]))
                first = next((i for i in range(n) if v[2][i] != ref[2][i]), n)
                raise CollectiveDivergence(
                    f"collective sequence of rank {r} ({v[1]} calls) diverges from rank 0 "
                    f"({ref[1]} calls) at call #{first}: rank0={ref[2][first] if first < len(ref[2]) else None} "
                    f"rank{r}={v[2][first] if first < len(v[2]) else None}")
        return ref[0]


_global = None


def maybe_enable():
    """Install a process-wide tracer when DDP_AMD_DEBUG=1; returns it (or None)."""
    global _global
    if os.environ.get("DDP_AMD_DEBUG", "0") not in ("0", "", "false") and _global is None:
        _global = CollectiveTracer().__enter__()
    return _global
