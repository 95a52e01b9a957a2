"""Plain-PyTorch fp32 reference implementations of every fused HIP op, in the
kernels' native layouts (NHWC activations, OHWI conv weights, [out][HW][C] fc
weight).  Used (a) as the numerics oracle of the GPU tests and (b) by nothing
on the GPU path - the HIP kernels are mandatory there (see ``ddp_amd.native``).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def bf16r(t: torch.Tensor) -> torch.Tensor:
    """Round to bf16 and back (what a bf16 activation store does)."""
    return t.to(torch.bfloat16).float()


def _f(t: torch.Tensor) -> torch.Tensor:
    """fp32 view of ``t`` - float64 stays float64 (the exact-fp32 path's oracle)."""
    return t if t.dtype == torch.float64 else t.float()


def nhwc_to_nchw(x):
    return x.permute(0, 3, 1, 2)


def nchw_to_nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


def conv1_relu(x: torch.Tensor, w_ohwi: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """x [B,H,W] fp32 -> NHWC fp32 relu(conv3x3(x)+b); w_ohwi [Cout,3,3,1]."""
    y = F.conv2d(x.unsqueeze(1), w_ohwi.permute(0, 3, 1, 2), b, padding=1)
    return nchw_to_nhwc(torch.relu(y))


def conv3x3(x_nhwc, w_ohwi, b, relu=True):
    y = F.conv2d(nhwc_to_nchw(x_nhwc), w_ohwi.permute(0, 3, 1, 2), b, padding=1)
    if relu:
        y = torch.relu(y)
    return nchw_to_nhwc(y)


def conv3x3_dgrad(dy_nhwc, w_ohwi):
    """dX of a 3x3/s1/p1 conv (NHWC in/out)."""
    dx = F.conv_transpose2d(nhwc_to_nchw(dy_nhwc), w_ohwi.permute(0, 3, 1, 2), padding=1)
    return nchw_to_nhwc(dx)


def conv3x3_wgrad(dy_nhwc, x_nhwc):
    """(dW OHWI, db) of a 3x3/s1/p1 conv."""
    x = _f(nhwc_to_nchw(x_nhwc))
    dy = _f(nhwc_to_nchw(dy_nhwc))
    cin, cout = x.shape[1], dy.shape[1]
    dw = torch.nn.grad.conv2d_weight(x, (cout, cin, 3, 3), dy, padding=1)
    return dw.permute(0, 2, 3, 1).contiguous(), dy.sum(dim=(0, 2, 3))


def conv1_wgrad(dz_nhwc, x):
    """(dW [Cout,3,3,1], db) of conv1 given its pre-activation gradient dZ (NHWC)."""
    dy = _f(nhwc_to_nchw(dz_nhwc))
    dw = torch.nn.grad.conv2d_weight(_f(x.unsqueeze(1)), (dy.shape[1], 1, 3, 3), dy, padding=1)
    return dw.permute(0, 2, 3, 1).contiguous(), dy.sum(dim=(0, 2, 3))


def fc_nhwc(x_nhwc, w_native, b):
    """logits = flatten_nhwc(x) @ w_native.reshape(out,-1).T + b."""
    B = x_nhwc.shape[0]
    return _f(x_nhwc.reshape(B, -1)) @ _f(w_native.reshape(w_native.shape[0], -1)).t() + b


def fc_bwd(dl, x_nhwc, w_native, mask=True):
    """(dX NHWC [masked by X>0], dW native) of fc_nhwc."""
    B = x_nhwc.shape[0]
    xf = _f(x_nhwc.reshape(B, -1))
    wf = _f(w_native.reshape(w_native.shape[0], -1))
    dx = dl @ wf
    if mask:
        dx = dx * (xf > 0)
    dw = dl.t() @ xf
    return dx.view_as(x_nhwc), dw.view_as(w_native)


def cross_entropy(logits, labels):
    """(mean loss, dlogits = (softmax - onehot)/B)."""
    lp = torch.log_softmax(_f(logits), dim=1)
    loss = F.nll_loss(lp, labels)
    d = lp.exp()
    d[torch.arange(logits.shape[0]), labels] -= 1.0
    return loss, d / logits.shape[0]


def simple_cnn_step_bf16(params: dict, x: torch.Tensor, labels: torch.Tensor, ws: int = 1):
    """fp32 PyTorch model of ONE SimpleCNN training step that rounds to bf16 at exactly
    the points the HIP pipeline stores bf16 (activations, MFMA operands, dZ tensors).

    ``params``: native layouts ``w1 [32,3,3,1]``, ``b1``, ``w2 [64,3,3,32]`` (OHWI),
    ``b2``, ``wfc [10,784,64]``, ``bfc``; ``x`` float [B,28,28] in [0,1].
    Returns (loss, grads dict in native layouts, prescaled by 1/ws).
    """
    B = x.shape[0]
    w1, b1, w2, b2 = params["w1"].float(), params["b1"].float(), params["w2"].float(), params["b2"].float()
    wfc, bfc = params["wfc"].float(), params["bfc"].float()
    w2b, wfcb = bf16r(w2), bf16r(wfc)
    a1 = bf16r(conv1_relu(x.float(), w1, b1))                      # [B,28,28,32]
    a2 = bf16r(conv3x3(a1, w2b, b2, relu=True))                     # [B,28,28,64]
    logits = fc_nhwc(a2, wfcb, bfc)
    loss, dl = cross_entropy(logits, labels)
    dz2 = bf16r((dl @ wfcb.reshape(wfcb.shape[0], -1)).view_as(a2) * (a2 > 0))
    dwfc = (dl.t() @ a2.reshape(B, -1)).view_as(wfc)
    dw2, db2 = conv3x3_wgrad(dz2, a1)
    dz1 = bf16r(conv3x3_dgrad(dz2, w2b)) * (a1 > 0)
    dw1, db1 = conv1_wgrad(dz1, x.float())
    s = 1.0 / ws
    return loss, {"w1": dw1 * s, "b1": db1 * s, "w2": dw2 * s, "b2": db2 * s,
                  "wfc": dwfc * s, "bfc": dl.sum(0) * s}


def simple_cnn_step_exact(params: dict, x: torch.Tensor, labels: torch.Tensor, ws: int = 1,
                          dtype: torch.dtype = torch.float64):
    """The same step without any bf16 rounding, evaluated in ``dtype`` (float64 by
    default): the oracle of the exact-fp32 path (``--dtype fp32``), whose MFMA results
    are plain fp32 fma chains.  Same arguments / returns as :func:`simple_cnn_step_bf16`."""
    B = x.shape[0]
    p = {k: v.to(dtype) for k, v in params.items()}
    w1, b1, w2, b2, wfc, bfc = p["w1"], p["b1"], p["w2"], p["b2"], p["wfc"], p["bfc"]
    x = x.to(dtype)
    a1 = conv1_relu(x, w1, b1)
    a2 = conv3x3(a1, w2, b2, relu=True)
    logits = fc_nhwc(a2, wfc, bfc)
    loss, dl = cross_entropy(logits, labels)
    dz2 = (dl @ wfc.reshape(wfc.shape[0], -1)).view_as(a2) * (a2 > 0)
    dwfc = (dl.t() @ a2.reshape(B, -1)).view_as(wfc)
    dw2, db2 = conv3x3_wgrad(dz2, a1)
    dz1 = conv3x3_dgrad(dz2, w2) * (a1 > 0)
    dw1, db1 = conv1_wgrad(dz1, x)
    s = 1.0 / ws
    return loss, {"w1": dw1 * s, "b1": db1 * s, "w2": dw2 * s, "b2": db2 * s,
                  "wfc": dwfc * s, "bfc": dl.sum(0) * s}
