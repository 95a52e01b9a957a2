"""SimpleCNN - the reference's only model family (reference model.py:4-20).

Topology (unchanged): Conv(1->32, 3x3, p1) -> ReLU -> Conv(32->64, 3x3, p1) ->
ReLU -> Flatten -> Linear(50176 -> 10); 520,586 parameters, no pooling / BN /
dropout.  Module tree and parameter names are the reference's (``net.0``,
``net.2``, ``fl``) so ``state_dict()`` (keys, shapes, ``_metadata``) is
identical; only the in-memory parameter layouts are native (see layers.py).

Forward dispatch:
* CUDA input -> the fused HIP autograd Functions (NHWC activations in
  ``compute_dtype``: bf16 by default, or fp32 for the reference's precision - exact
  fp32 MFMA conv2; fused bias+ReLU epilogues, split-K fc) - ``ops/functional.py``;
* CPU input  -> plain fp32 PyTorch ops in the reference's NCHW order.
The training engine (``engine/fused_step.py``) drives the same parameters with
an even more fused kernel chain and never calls ``forward``.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .layers import Conv2d, Linear

H = W = 28
C1, C2, NCLS = 32, 64, 10


class SimpleCNN(nn.Module):
    def __init__(self, num_classes: int = NCLS, compute_dtype: torch.dtype = torch.bfloat16):
        super().__init__()
        if compute_dtype not in (torch.bfloat16, torch.float32):
            raise ValueError("compute_dtype must be torch.bfloat16 or torch.float32")
        self.compute_dtype = compute_dtype
        self.net = nn.Sequential(
            Conv2d(1, C1, 3, padding=1),
            nn.ReLU(),
            Conv2d(C1, C2, 3, padding=1),
            nn.ReLU(),
            nn.Flatten(),
        )
        self.fl = Linear(C2 * H * W, num_classes, in_layout=(C2, H, W))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if x.is_cuda:
            from ..ops import functional as Fh

            dt = self.compute_dtype
            a1 = Fh.conv1_relu(x, self.net[0].weight, self.net[0].bias, dt)
            a2 = Fh.conv3x3_relu(a1, self.net[2].weight, self.net[2].bias, True, dt)
            return Fh.linear_nhwc(a2, self.fl.weight, self.fl.bias, dt)
        h = torch.relu(self.net[0].forward_nchw(x))
        h = torch.relu(self.net[2].forward_nchw(h))
        return self.fl(torch.flatten(h, 1))


def reference_simple_cnn() -> nn.Module:
    """The reference architecture built from stock ``torch.nn`` layers (test oracle only)."""
    m = nn.Module()
    m.net = nn.Sequential(nn.Conv2d(1, C1, 3, padding=1), nn.ReLU(),
                          nn.Conv2d(C1, C2, 3, padding=1), nn.ReLU(), nn.Flatten())
    m.fl = nn.Linear(C2 * H * W, NCLS)
    m.forward = lambda x: m.fl(m.net(x))
    return m


def param_count(model: nn.Module) -> int:
    return sum(p.numel() for p in model.parameters())
