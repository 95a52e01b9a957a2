"""Layers that keep MI355X-native parameter layouts but speak the reference's state_dict.

Native layouts (what the gfx950 kernels read):

* ``Conv2d.weight``: **OHWI** ``[Cout, KH, KW, Cin]`` - the implicit-GEMM K axis
  (tap, ci) is contiguous, matching NHWC activations.
* ``Linear.weight`` with ``in_layout=(C, H, W)``: ``[out, H*W, C]`` - the
  activation's NHWC memory order, so the fc kernels stream it contiguously.

The checkpoint contract is the reference's (``model.py:8-16`` + ``torch.save`` of
``model.module.state_dict()``): OIHW conv weights and an
NCHW-flatten ``[out, C*H*W]`` fc weight.  ``_save_to_state_dict`` /
``_load_from_state_dict`` permute between the two, so ``state_dict()`` keys,
shapes, ``_metadata`` and values are exactly what the reference writes, and a
reference checkpoint loads into this model unchanged.

Initialisation draws from the RNG exactly like ``torch.nn.Conv2d``/``Linear``
(kaiming-uniform a=sqrt(5) on the reference-shaped tensor, then the bias), so
``torch.manual_seed(s)`` gives bitwise the same initial weights as the
reference model.
"""
from __future__ import annotations

import math
from typing import Iterable

import torch
import torch.nn as nn
import torch.nn.functional as F


def _canonical(t: torch.Tensor) -> torch.Tensor:
    """Fresh tensor with its own storage and canonical row-major strides (incl. size-1
    dims), so ``torch.save`` writes exactly the bytes a stock nn layer would."""
    return t.clone(memory_format=torch.contiguous_format)


def _kaiming_uniform_ref(shape, fan_in) -> torch.Tensor:
    w = torch.empty(shape)
    nn.init.kaiming_uniform_(w, a=math.sqrt(5))
    return w


def _bias_uniform(n, fan_in) -> torch.Tensor:
    b = torch.empty(n)
    bound = 1.0 / math.sqrt(fan_in) if fan_in > 0 else 0.0
    nn.init.uniform_(b, -bound, bound)
    return b


class Conv2d(nn.Module):
    """2-D convolution with an OHWI (channels-last) weight; reference-layout state_dict."""

    def __init__(self, in_channels: int, out_channels: int, kernel_size: int, stride: int = 1,
                 padding: int = 0, bias: bool = True):
        super().__init__()
        self.in_channels, self.out_channels = in_channels, out_channels
        self.kernel_size, self.stride, self.padding = kernel_size, stride, padding
        k = kernel_size
        fan_in = in_channels * k * k
        w_ref = _kaiming_uniform_ref((out_channels, in_channels, k, k), fan_in)
        self.weight = nn.Parameter(w_ref.permute(0, 2, 3, 1).contiguous())
        self.bias = nn.Parameter(_bias_uniform(out_channels, fan_in)) if bias else None

    # reference (OIHW) view of the native weight; shares memory
    def weight_oihw(self) -> torch.Tensor:
        return self.weight.permute(0, 3, 1, 2)

    def forward_nchw(self, x: torch.Tensor) -> torch.Tensor:
        """Plain PyTorch forward on NCHW fp32 (CPU reference path)."""
        return F.conv2d(x, self.weight_oihw(), self.bias, self.stride, self.padding)

    def forward(self, x):
        return self.forward_nchw(x)

    def _save_to_state_dict(self, destination, prefix, keep_vars):
        w = self.weight_oihw()
        destination[prefix + "weight"] = _canonical(w if keep_vars else w.detach())
        if self.bias is not None:
            b = self.bias
            destination[prefix + "bias"] = _canonical(b if keep_vars else b.detach())

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys,
                              unexpected_keys, error_msgs):
        for name in ("weight", "bias"):
            key = prefix + name
            p = getattr(self, name)
            if p is None:
                continue
            if key not in state_dict:
                missing_keys.append(key)
                continue
            v = state_dict[key]
            if name == "weight":
                exp = (self.out_channels, self.in_channels, self.kernel_size, self.kernel_size)
                if tuple(v.shape) != exp:
                    error_msgs.append(f"size mismatch for {key}: copying a param with shape "
                                      f"{tuple(v.shape)}, the shape in current model is {exp}.")
                    continue
                v = v.permute(0, 2, 3, 1)
            elif tuple(v.shape) != tuple(p.shape):
                error_msgs.append(f"size mismatch for {key}: {tuple(v.shape)} vs {tuple(p.shape)}")
                continue
            with torch.no_grad():
                p.copy_(v)
        if strict:
            for k in state_dict:
                if k.startswith(prefix) and k[len(prefix):] not in ("weight", "bias") and "." not in k[len(prefix):]:
                    unexpected_keys.append(k)

    def extra_repr(self):
        return (f"{self.in_channels}, {self.out_channels}, kernel_size={self.kernel_size}, "
                f"stride={self.stride}, padding={self.padding}, layout=OHWI")


class Linear(nn.Module):
    """Linear layer; with ``in_layout=(C,H,W)`` it consumes NHWC-flattened activations.

    Reference semantics: ``y = x_nchw_flat @ W_ref.T + b`` with ``W_ref [out, C*H*W]``.
    Native weight: ``[out, H*W, C]`` (== W_ref permuted), so that
    ``y = x_nhwc_flat @ W_native.reshape(out,-1).T + b`` is the same function.
    """

    def __init__(self, in_features: int, out_features: int, bias: bool = True,
                 in_layout: tuple[int, int, int] | None = None):
        super().__init__()
        self.in_features, self.out_features = in_features, out_features
        self.in_layout = in_layout
        w_ref = _kaiming_uniform_ref((out_features, in_features), in_features)
        if in_layout is not None:
            C, H, W = in_layout
            assert C * H * W == in_features, "in_layout does not match in_features"
            w = w_ref.view(out_features, C, H * W).permute(0, 2, 1).contiguous()
        else:
            w = w_ref
        self.weight = nn.Parameter(w)
        self.bias = nn.Parameter(_bias_uniform(out_features, in_features)) if bias else None

    def weight_ref(self) -> torch.Tensor:
        """Reference-layout ``[out, C*H*W]`` view/copy of the weight (differentiable)."""
        if self.in_layout is None:
            return self.weight
        C, H, W = self.in_layout
        return self.weight.permute(0, 2, 1).reshape(self.out_features, C * H * W)

    def forward(self, x):  # x in reference (NCHW-flatten) order
        return F.linear(x, self.weight_ref(), self.bias)

    def _save_to_state_dict(self, destination, prefix, keep_vars):
        w = self.weight_ref()
        destination[prefix + "weight"] = _canonical(w if keep_vars else w.detach())
        if self.bias is not None:
            b = self.bias
            destination[prefix + "bias"] = _canonical(b if keep_vars else b.detach())

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys,
                              unexpected_keys, error_msgs):
        for name in ("weight", "bias"):
            key = prefix + name
            p = getattr(self, name)
            if p is None:
                continue
            if key not in state_dict:
                missing_keys.append(key)
                continue
            v = state_dict[key]
            if name == "weight":
                exp = (self.out_features, self.in_features)
                if tuple(v.shape) != exp:
                    error_msgs.append(f"size mismatch for {key}: copying a param with shape "
                                      f"{tuple(v.shape)}, the shape in current model is {exp}.")
                    continue
                if self.in_layout is not None:
                    C, H, W = self.in_layout
                    v = v.view(self.out_features, C, H * W).permute(0, 2, 1)
            elif tuple(v.shape) != tuple(p.shape):
                error_msgs.append(f"size mismatch for {key}: {tuple(v.shape)} vs {tuple(p.shape)}")
                continue
            with torch.no_grad():
                p.copy_(v)

    def extra_repr(self):
        lay = f", in_layout=NHWC{self.in_layout}" if self.in_layout else ""
        return f"in_features={self.in_features}, out_features={self.out_features}{lay}"


# ----------------------------------------------------------------------------- flat storage
class FlatSpace:
    """One contiguous fp32 buffer that every parameter of a module is a view into.

    ``order`` lists parameters in gradient-ready order (reverse registration by
    default, which is the order autograd produces SimpleCNN's gradients); each
    parameter starts on a ``align``-element (256 B) boundary.  A twin buffer holds
    the gradients, and ``param.grad`` is set to the matching view so autograd
    accumulates in place (DDP buckets are then plain slices: no pack/unpack).
    """

    def __init__(self, module: nn.Module, align: int = 64, order: Iterable[str] | None = None):
        named = dict(module.named_parameters())
        names = list(order) if order is not None else list(reversed(list(named.keys())))
        if sorted(names) != sorted(named.keys()):
            raise ValueError("FlatSpace order must list every parameter exactly once")
        dev = next(iter(named.values())).device
        self.names = names
        self.offsets, self.numels, self.shapes = {}, {}, {}
        off = 0
        for n in names:
            p = named[n]
            self.offsets[n] = off
            self.numels[n] = p.numel()
            self.shapes[n] = tuple(p.shape)
            off += (p.numel() + align - 1) // align * align
        self.numel = off
        self.device = dev
        self.params = torch.zeros(off, dtype=torch.float32, device=dev)
        self.grads = torch.zeros(off, dtype=torch.float32, device=dev)
        self.module = module
        # re-home every parameter into the flat buffer (same Parameter object identity is
        # not preserved; optimizers must be built after flattening)
        for n in names:
            mod, attr = _resolve(module, n)
            old = getattr(mod, attr)
            view = self.view(self.params, n)
            with torch.no_grad():
                view.copy_(old.detach())
            newp = nn.Parameter(view, requires_grad=old.requires_grad)
            gview = self.view(self.grads, n)
            if old.grad is not None:
                with torch.no_grad():
                    gview.copy_(old.grad)
            newp.grad = gview
            newp._ddp_amd_fs = self  # kernels find the bf16 weight copy through this
            mod._parameters[attr] = newp
        module._ddp_amd_flat = self
        self._bf16 = None
        self._bf16_version = -1
        self._pad4: dict = {}  # flat offset -> bf16 [..][4] copy of a [..][3] parameter

    def bf16_params(self) -> torch.Tensor:
        """bf16 copy of the flat parameters (the MFMA kernels' weight operand).

        FusedSGD rewrites it inside its update kernel (a SHADOW_BF16 region over the whole
        buffer), so a training step never converts weights; any other write to the fp32
        parameters goes through torch ops, which bump the flat buffer's version counter
        (shared by every parameter view), and the copy is rebuilt on the next call."""
        if self._bf16 is None:
            self._bf16 = torch.empty(self.numel, dtype=torch.bfloat16, device=self.device)
        if self._bf16_version != self.params._version:
            with torch.no_grad():
                self._bf16.copy_(self.params)
                for off, buf in self._pad4.items():
                    self._fill_pad4(off, buf)
            self._bf16_version = self.params._version
        return self._bf16

    def _fill_pad4(self, off: int, buf: torch.Tensor):
        n = buf.numel() // 4 * 3
        buf.view(-1, 4)[:, :3].copy_(self.params[off:off + n].view(-1, 3))

    def bf16_pad4_view(self, p: torch.Tensor):
        """bf16 copy of a ``[..., 3]`` parameter zero-padded to ``[..., 4]`` (the ResNet stem
        weight as its conv kernel loads it), kept fresh exactly like :meth:`bf16_params`:
        FusedSGD rewrites it in its update pass (a SHADOW_BF16_PAD4 region) and any other
        write rebuilds it with the flat copy.  ``None`` if ``p`` is not a flat-space view."""
        if p.shape[-1] != 3 or self.bf16_view(p) is None:  # bf16_view also refreshes
            return None
        off = (p.data_ptr() - self.params.data_ptr()) // self.params.element_size()
        buf = self._pad4.get(off)
        if buf is None:
            buf = torch.zeros(*p.shape[:-1], 4, dtype=torch.bfloat16, device=self.device)
            with torch.no_grad():
                self._fill_pad4(off, buf)
            self._pad4[off] = buf
        return buf

    def pad4_shadows(self) -> list:
        """SGD shadow regions (off, n, dst, kind=4, 0, 0, 0) of the padded copies."""
        return [(off, buf.numel() // 4 * 3, buf, 4, 0, 0, 0) for off, buf in self._pad4.items()]

    def bf16_view(self, p: torch.Tensor):
        """The bf16 copy of parameter ``p``, same shape; ``None`` if ``p`` no longer lives
        in this flat space (e.g. its ``.data`` was replaced) or is not contiguous."""
        es = self.params.element_size()
        off, rem = divmod(p.data_ptr() - self.params.data_ptr(), es)
        if rem or off < 0 or off + p.numel() > self.numel or not p.is_contiguous() or p.dtype != torch.float32:
            return None
        return self.bf16_params()[off:off + p.numel()].view(p.shape)

    def params_written(self):
        """The fp32 parameters were rewritten outside torch's in-place tracking (a c10d /
        RCCL broadcast writes the storage without bumping the version counter): rebuild the
        bf16 copies on next use."""
        self._bf16_version = -1

    def mark_bf16_fresh(self):
        """Called by the optimizer after a step that rewrote the bf16 copy."""
        if self._bf16 is not None:
            self._bf16_version = self.params._version

    def view(self, buf: torch.Tensor, name: str) -> torch.Tensor:
        o, n = self.offsets[name], self.numels[name]
        return buf[o:o + n].view(self.shapes[name])

    def param(self, name):
        mod, attr = _resolve(self.module, name)
        return getattr(mod, attr)

    def reattach_grads(self):
        """Point every ``.grad`` back at its flat view (after a set_to_none zero_grad)."""
        pairs = getattr(self, "_pairs", None)  # cached; rebuilt if the first parameter was replaced
        if pairs is None or self.param(self.names[0]) is not pairs[0][0]:
            pairs = self._pairs = [(self.param(n), self.view(self.grads, n)) for n in self.names]
        for p, g in pairs:
            if p.grad is None:
                p.grad = g
            elif p.grad.data_ptr() != g.data_ptr():
                g.copy_(p.grad)
                p.grad = g

    def zero_grad(self, lazy: bool = False):
        """Zero every gradient.  ``lazy`` (FusedSGD): skip the memset when every parameter's
        gradient was written by a direct producer last step (ops/direct_grad.py lazy_zero)."""
        from ..ops import direct_grad

        if lazy:
            self.reattach_grads()
            if direct_grad.lazy_zero(p for p, _ in self._pairs):
                return
            self.grads.zero_()
            return
        self.grads.zero_()
        self.reattach_grads()
        for p, _ in self._pairs:  # (zeroed for real: nothing fresh, nothing written yet)
            direct_grad._fresh.discard(p)
            direct_grad._written.discard(p)


class BufferSpace:
    """Every buffer of a module (BatchNorm running stats, ``num_batches_tracked``, ...) as a
    view into one contiguous flat tensor PER DTYPE, so DDP's ``broadcast_buffers`` is one
    collective per dtype per forward (2 for BatchNorm models: float32 stats, int64 counters)
    instead of one per tensor (torch DDP coalesces the same way,
    ``torch/nn/parallel/distributed.py:1557-1558``; ResNet-18 has 60 buffers).

    Each flat tensor has the dtype of its buffers, so ``torch.save(module.state_dict())``
    sees only same-typed views of each storage (one byte buffer shared by float32 and int64
    views made it refuse: "Cannot save multiple tensors or storages that view the same data
    as different types" - ADVICE r2).  Each buffer starts on a 64-byte boundary; the
    module's ``_buffers`` entries are replaced by views, so in-place kernel updates land in
    the flat tensors.  :meth:`rehome` copies back any buffer that was REPLACED by a new
    tensor of the same dtype / shape / device (``module.buf = t``); :func:`buffer_space`
    rebuilds the space when a buffer changed dtype, shape or device (``model.to(...)``,
    ``.double()``) instead of silently copying it back."""

    def __init__(self, module: nn.Module, align: int = 64):
        self.module = module
        self.names = [n for n, _ in module.named_buffers()]
        named = dict(module.named_buffers())
        self.offsets, self.meta = {}, {}
        totals = {}  # dtype -> elements
        for n in self.names:
            b = named[n]
            es = b.element_size()
            q = max(1, align // es)  # elements per alignment quantum
            off = totals.get(b.dtype, 0)
            self.offsets[n] = off
            self.meta[n] = (b.dtype, tuple(b.shape), b.device)
            totals[b.dtype] = off + (b.numel() + q - 1) // q * q
        dev = named[self.names[0]].device if self.names else torch.device("cpu")
        self.flats = {dt: torch.zeros(max(n, 1), dtype=dt, device=dev) for dt, n in totals.items()}
        self._views = {}
        for n in self.names:
            v = self.view(n)
            with torch.no_grad():
                v.copy_(named[n])
            self._views[n] = v
            mod, attr = _resolve(module, n)
            mod._buffers[attr] = v
        module._ddp_amd_bufs = self

    def flat_list(self) -> list:
        """The flat tensors, in first-appearance order of their dtypes (one collective each)."""
        return list(self.flats.values())

    def view(self, name: str) -> torch.Tensor:
        """Alias of the buffer's elements with its OWN version counter (``set_`` on the
        storage, not an autograd view): BatchNorm saves running stats for backward, and
        a version counter shared by all 60 buffers would make every later layer's
        in-place stat update look like a modification of the saved tensor."""
        dt, shape, _ = self.meta[name]
        flat = self.flats[dt]
        t = torch.empty(0, dtype=dt, device=flat.device)
        t.set_(flat.untyped_storage(), self.offsets[name], shape)
        return t

    def matches(self) -> bool:
        """Whether every current buffer still has the dtype / shape / device it was laid
        out with (and no buffer was added or removed)."""
        cur = dict(self.module.named_buffers())
        if list(cur) != self.names:
            return False
        return all((b.dtype, tuple(b.shape), b.device) == self.meta[n] for n, b in cur.items())

    def rehome(self) -> int:
        """Pull replaced buffers back into the flat tensors; returns how many moved.
        Raises if a replacement changed dtype / shape / device (use :func:`buffer_space`,
        which rebuilds the space in that case)."""
        moved = 0
        for n in self.names:
            mod, attr = _resolve(self.module, n)
            cur, v = mod._buffers.get(attr), self._views[n]
            if cur is None or cur.data_ptr() == v.data_ptr():
                continue
            if (cur.dtype, tuple(cur.shape), cur.device) != self.meta[n]:
                raise RuntimeError(f"buffer {n} changed dtype/shape/device: rebuild the BufferSpace")
            with torch.no_grad():
                v.copy_(cur)
            mod._buffers[attr] = v
            moved += 1
        return moved


def buffer_space(module: nn.Module) -> BufferSpace | None:
    """The module's BufferSpace (created on first use, rebuilt when a buffer changed dtype,
    shape or device); ``None`` if it has no buffers."""
    bs = getattr(module, "_ddp_amd_bufs", None)
    if bs is None or not bs.matches():
        if not any(True for _ in module.buffers()):
            return None
        bs = BufferSpace(module)
    bs.rehome()
    return bs


def _resolve(module: nn.Module, name: str):
    parts = name.split(".")
    mod = module
    for p in parts[:-1]:
        mod = getattr(mod, p)
    return mod, parts[-1]


def flat_space(module: nn.Module, **kw) -> FlatSpace:
    """Return the module's FlatSpace, creating it (on the module's device) if needed."""
    fs = getattr(module, "_ddp_amd_flat", None)
    if fs is not None:
        cur = dict(module.named_parameters())
        ok = all(cur[n].data_ptr() == fs.view(fs.params, n).data_ptr() for n in fs.names)
        dev_ok = all(cur[n].device == fs.device for n in fs.names)
        if ok and dev_ok:
            return fs
    return FlatSpace(module, **kw)
