"""Direct gradient accumulation for the module path's HIP autograd Functions.

Autograd's default contract is "a Function returns its input gradients, AccumulateGrad
adds them into ``param.grad``": for a flat-space parameter that is one more pass over
every weight gradient per step (an add kernel per parameter, 62 for ResNet-18).  Here a
Function whose weight gradient is produced by a reduction kernel (conv wgrad split-K
reduce, BatchNorm strip reduce, the fc GEMM) accumulates straight into ``param.grad`` -
the flat gradient view FlatSpace attaches - and returns ``None`` for that input.

The parameter's AccumulateGrad node still runs when its incoming gradient is undefined,
and it fires the post-accumulate-grad hooks (DDP's bucket-ready hook) all the same -
``tests/test_direct_grad_cpu.py`` pins that engine behaviour, which the protocol relies on.

Used only when ``param.grad`` exists as a contiguous fp32 tensor and the backward does
not build a graph (``create_graph=False``).  ``torch.autograd.grad(...)`` callers - who
must not see ``.grad`` written - wrap the call in :func:`disabled`.
"""
from __future__ import annotations

import contextlib
import weakref

import torch

_enabled = True

# Lazy zeroing (FusedSGD.zero_grad -> FlatSpace.zero_grad(lazy=True)).  When every parameter
# of a flat space was written by a direct producer during the previous backward, zero_grad
# skips the memset of the whole gradient buffer (a fill kernel inside every captured
# ResNet-18 step: 47 MB, ~8.5 us, profiles/r6_resnet) and marks the parameters fresh: the
# first producer write of the step then overwrites (beta = 0) instead of adding.  A fresh
# parameter whose gradient takes the autograd path instead is zeroed before AccumulateGrad
# adds into it (grad_dst), and one nobody wrote is zeroed before the optimizer reads it
# (flush_fresh).
class _TensorSet:
    """A set of tensors by identity (a WeakSet would compare tensors with ``==``)."""

    def __init__(self):
        self._d: dict[int, weakref.ref] = {}

    def __contains__(self, p) -> bool:
        r = self._d.get(id(p))
        return r is not None and r() is p

    def add(self, p):
        self._d[id(p)] = weakref.ref(p)

    def discard(self, p):
        if p in self:
            del self._d[id(p)]


_fresh = _TensorSet()
_written = _TensorSet()


@contextlib.contextmanager
def disabled():
    global _enabled
    old, _enabled = _enabled, False
    try:
        yield
    finally:
        _enabled = old


def grad_dst(p: torch.Tensor):
    """``p.grad`` if the backward may accumulate into it directly, else ``None``."""
    if not _enabled or torch.is_grad_enabled() or not p.requires_grad:
        _unfresh(p)
        return None
    g = p.grad
    if g is None or g.dtype != torch.float32 or not g.is_contiguous() or g.shape != p.shape:
        _unfresh(p)
        return None
    return g


def _unfresh(p: torch.Tensor):
    if p in _fresh:
        _fresh.discard(p)
        if p.grad is not None:
            p.grad.zero_()


def accumulate(p: torch.Tensor) -> bool:
    """For a producer about to write ``p.grad`` (from :func:`grad_dst`): True - add into it;
    False - overwrite it (its first write after a lazy zero_grad)."""
    _written.add(p)
    if p in _fresh:
        _fresh.discard(p)
        return False
    return True


def lazy_zero(params) -> bool:
    """FlatSpace.zero_grad(lazy=True): True (and the parameters marked fresh) when every one
    was written by a direct producer since the last zero_grad; False: memset as usual."""
    params = list(params)
    ok = bool(params) and all(p in _written for p in params)
    for p in params:
        _written.discard(p)
        if ok:
            _fresh.add(p)
        else:
            _fresh.discard(p)
    return ok


def flush_fresh(params):
    """Zero the gradient of every parameter still fresh (no producer wrote it this step)."""
    for p in params:
        _unfresh(p)
