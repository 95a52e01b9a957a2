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

import torch

_enabled = True


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
        return None
    g = p.grad
    if g is None or g.dtype != torch.float32 or not g.is_contiguous() or g.shape != p.shape:
        return None
    return g
