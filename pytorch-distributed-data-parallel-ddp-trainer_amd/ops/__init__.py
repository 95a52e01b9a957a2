"""Ops library: HIP-kernel autograd Functions (GPU) with fp32 PyTorch references (CPU/tests)."""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import reference
from .sgd import FusedSGD


class CrossEntropyLoss(nn.Module):
    """``nn.CrossEntropyLoss()`` (mean) - fused HIP softmax-xent on the GPU.

    Reference: train_ddp.py:40 ``loss_fn = nn.CrossEntropyLoss()``.
    """

    def forward(self, logits: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
        if logits.is_cuda:
            from .functional import cross_entropy

            return cross_entropy(logits, labels)
        return F.cross_entropy(logits, labels)


__all__ = ["CrossEntropyLoss", "FusedSGD", "reference"]
