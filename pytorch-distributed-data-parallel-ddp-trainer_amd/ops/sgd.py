"""Flat-buffer SGD with ``torch.optim.SGD`` semantics and state_dict format.

Reference: ``optim.SGD(model.parameters(), lr=0.01)`` (train_ddp.py:41) and
``opt.step()`` (train_ddp.py:200).  On the GPU one HIP kernel (``sgd_kernel`` in
csrc/kernels/optim.hip) updates the whole flat parameter buffer of the model
(weight decay / momentum / dampening / nesterov / maximize as in
torch/optim/sgd.py ``_single_tensor_sgd``) and refreshes any registered bf16
shadow copies in the same pass.  On the CPU the identical math runs as torch ops
over the same flat buffers.

``state_dict()`` reproduces ``torch.optim.SGD.state_dict()`` exactly (same
``param_groups`` keys and order, ``params`` = registration-order indices, and
``momentum_buffer`` tensors in the reference layout), so checkpoints stay
byte-compatible with the reference.
"""
from __future__ import annotations

import torch

from ..models.layers import FlatSpace, flat_space

_DEFAULTS = dict(lr=1e-3, momentum=0, dampening=0, weight_decay=0, nesterov=False,
                 maximize=False, foreach=None, differentiable=False, fused=None)


class FusedSGD:
    def __init__(self, model: torch.nn.Module, lr: float = 1e-3, momentum: float = 0,
                 dampening: float = 0, weight_decay: float = 0, nesterov: bool = False,
                 maximize: bool = False):
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        self.model = model
        self.flat: FlatSpace = flat_space(model)
        g = dict(_DEFAULTS)
        g.update(lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                 nesterov=nesterov, maximize=maximize)
        self.param_groups = [g]
        self._reg_names = [n for n, _ in model.named_parameters()]
        self.momentum_buffer: torch.Tensor | None = None
        self.shadows: list[tuple] = []  # (off, n, bf16 dst, kind, a, b, c)
        self.steps = 0

    # ------------------------------------------------------------------ API
    @property
    def lr(self):
        return self.param_groups[0]["lr"]

    def zero_grad(self, set_to_none: bool = True):
        # grads are views of the flat buffer: "none" is a memset that keeps the views - or no
        # memset at all when every gradient's producer overwrites it (direct_grad lazy zeroing)
        self.flat.zero_grad(lazy=True)

    @torch.no_grad()
    def step(self):
        g = self.param_groups[0]
        fs = self.flat
        fs.reattach_grads()
        from . import direct_grad

        direct_grad.flush_fresh(p for p, _ in fs._pairs)
        first = self.momentum_buffer is None
        if g["momentum"] != 0 and first:
            self.momentum_buffer = torch.zeros_like(fs.params)
        if fs.params.is_cuda:
            from .. import native

            shadows = self.shadows
            if fs._bf16 is not None:  # the model's bf16 weight copy, refreshed in the same pass
                shadows = shadows + [(0, fs.numel, fs._bf16, 1, 0, 0, 0)] + fs.pad4_shadows()
            native.require().sgd(fs.params, fs.grads, self.momentum_buffer, g["lr"], g["momentum"],
                                 g["dampening"], g["weight_decay"], g["nesterov"], g["maximize"],
                                 first, True, shadows)
            fs.mark_bf16_fresh()
        else:
            self._step_torch(first)
        self.steps += 1

    def _step_torch(self, first: bool):
        g = self.param_groups[0]
        p, d = self.flat.params, self.flat.grads
        d = -d if g["maximize"] else d.clone()
        if g["weight_decay"] != 0:
            d = d.add(p, alpha=g["weight_decay"])
        if g["momentum"] != 0:
            buf = self.momentum_buffer
            if first:
                buf.copy_(d)
            else:
                buf.mul_(g["momentum"]).add_(d, alpha=1 - g["dampening"])
            d = d.add(buf, alpha=g["momentum"]) if g["nesterov"] else buf
        p.add_(d, alpha=-g["lr"])

    # ------------------------------------------------------------------ state
    def state_dict(self):
        state = {}
        if self.momentum_buffer is not None:
            ref = _to_reference_layout(self.model, self.flat, self.momentum_buffer)
            for i, n in enumerate(self._reg_names):
                state[i] = {"momentum_buffer": ref[n]}
        groups = []
        for g in self.param_groups:
            d = {k: g[k] for k in _DEFAULTS}
            d["params"] = list(range(len(self._reg_names)))
            groups.append(d)
        return {"state": state, "param_groups": groups}

    def load_state_dict(self, sd):
        groups = sd["param_groups"]
        if len(groups) != 1 or len(groups[0]["params"]) != len(self._reg_names):
            raise ValueError("optimizer state_dict does not match this model")
        for k in _DEFAULTS:
            if k in groups[0]:
                self.param_groups[0][k] = groups[0][k]
        st = sd.get("state", {})
        if st:
            buf = torch.zeros_like(self.flat.params)
            ref = {self._reg_names[int(i)]: v["momentum_buffer"] for i, v in st.items()
                   if "momentum_buffer" in v}
            _from_reference_layout(self.model, self.flat, ref, buf)
            self.momentum_buffer = buf
            # torch only creates a momentum buffer in its first step: a loaded buffer means
            # the next step is a regular update (buf = m*buf + (1-d)*g), never the
            # initialisation step (buf = g) - the fused engine keys that off ``steps``
            self.steps = max(self.steps, 1)
        else:
            self.momentum_buffer = None
            self.steps = 0

    def mark_started(self):
        """A momentum buffer arrived from elsewhere (resume broadcast): treat as started."""
        if self.momentum_buffer is not None:
            self.steps = max(self.steps, 1)


def _owner(model, name):
    mod = model
    for p in name.split(".")[:-1]:
        mod = getattr(mod, p)
    return mod, name.split(".")[-1]


def _to_reference_layout(model, fs: FlatSpace, flat_buf: torch.Tensor) -> dict:
    """Per-parameter tensors of ``flat_buf`` in the layout the reference state_dict uses."""
    from ..models.layers import Conv2d, Linear

    out = {}
    for n in fs.names:
        v = fs.view(flat_buf, n).detach()
        mod, attr = _owner(model, n)
        if attr == "weight" and isinstance(mod, Conv2d):
            v = v.permute(0, 3, 1, 2)
        elif attr == "weight" and isinstance(mod, Linear) and mod.in_layout is not None:
            C, H, W = mod.in_layout
            v = v.permute(0, 2, 1).reshape(mod.out_features, C * H * W)
        out[n] = v.contiguous().clone()
    return out


def _from_reference_layout(model, fs: FlatSpace, ref: dict, flat_buf: torch.Tensor):
    from ..models.layers import Conv2d, Linear

    for n, v in ref.items():
        mod, attr = _owner(model, n)
        if attr == "weight" and isinstance(mod, Conv2d):
            v = v.permute(0, 2, 3, 1)
        elif attr == "weight" and isinstance(mod, Linear) and mod.in_layout is not None:
            C, H, W = mod.in_layout
            v = v.reshape(mod.out_features, C, H * W).permute(0, 2, 1)
        fs.view(flat_buf, n).copy_(v)
