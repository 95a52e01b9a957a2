"""The direct-gradient protocol of the module path (ops/direct_grad.py), on the CPU.

The HIP Functions accumulate weight gradients straight into ``param.grad`` and return
None; DDP's bucket-ready hook must still fire exactly once per parameter per backward.
That relies on autograd running the parameter's AccumulateGrad node (and its
post-accumulate hooks) for an undefined incoming gradient - pinned here so a torch
upgrade that changes it fails loudly instead of hanging a bucket.
"""
import torch

from ddp_amd.ops import direct_grad


class _DirectMul(torch.autograd.Function):
    """y = x * w, dw accumulated in place when allowed (the resnet_fn pattern)."""

    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x)
        ctx.w = w
        return x * w.detach()

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        dst = direct_grad.grad_dst(ctx.w)
        dw = (g * x).sum(0)
        if dst is not None:
            dst.add_(dw)
            return g * ctx.w.detach(), None
        return g * ctx.w.detach(), dw


def test_post_accumulate_hook_fires_once_for_direct_gradient():
    w = torch.nn.Parameter(torch.ones(3))
    w.grad = torch.zeros(3)
    calls = []
    w.register_post_accumulate_grad_hook(lambda p: calls.append(p.grad.clone()))
    x = torch.randn(4, 3)
    _DirectMul.apply(x, w).sum().backward()
    assert len(calls) == 1
    assert torch.allclose(calls[0], x.sum(0))
    _DirectMul.apply(x, w).sum().backward()  # accumulation, like a second micro-batch
    assert len(calls) == 2 and torch.allclose(w.grad, 2 * x.sum(0))


def test_direct_gradient_fallbacks():
    w = torch.nn.Parameter(torch.ones(3))
    x = torch.randn(4, 3)
    _DirectMul.apply(x, w).sum().backward()  # no .grad yet: returned, AccumulateGrad stores it
    assert torch.allclose(w.grad, x.sum(0))
    w.grad = None
    with direct_grad.disabled():
        (gw,) = torch.autograd.grad(_DirectMul.apply(x, w).sum(), [w])
    assert torch.allclose(gw, x.sum(0)) and w.grad is None
