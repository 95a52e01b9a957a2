"""HIP autograd Functions for ResNet-style networks (NHWC bf16 activations).

==================  ================================================  ===========================================
Function            forward kernels                                   backward kernels
==================  ================================================  ===========================================
conv_bn_act         conv_gemm_fwd (+ fused BN sum/sumsq epilogue),    bn_bwd_reduce -> grad_reduce -> bn_bwd_apply,
                    bn_finalize (running stats), bn_apply             conv_gemm_dgrad (transposed weight),
                    (+ residual add + ReLU)                           conv_gemm_wgrad -> grad_reduce
maxpool3x3s2        maxpool_fwd (argmax saved)                        maxpool_bwd (deterministic gather)
global_avgpool      avgpool_fwd                                       avgpool_bwd
linear_head         sgemm (+bias)                                     sgemm x2 (dX, dW), bias = sum
==================  ================================================  ===========================================

Weights are fp32 OHWI masters converted to bf16 per call (the stem's 3 input
channels are zero-padded to 4 so its K-steps pack 8 taps x 4 channels).
"""
from __future__ import annotations

import torch

from .. import native

BF16 = torch.bfloat16


def _C():
    return native.require()


def _wgrad_ppc(P: int, gx: int, gy: int, target_blocks: int = 1024) -> int:
    chunks = max(1, target_blocks // max(1, gx * gy))
    ppc = -(-P // chunks)
    return max(32, -(-ppc // 32) * 32)


def to_nhwc4(x: torch.Tensor) -> torch.Tensor:
    """NCHW float image batch -> NHWC bf16 with channels zero-padded to 4 (stem input)."""
    n, c, h, w = x.shape
    out = torch.zeros(n, h, w, 4, dtype=BF16, device=x.device)
    out[..., :c] = x.permute(0, 2, 3, 1)
    return out


class _ConvBNAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, gamma, beta, running_mean, running_var, res, stride, pad, relu,
                training, momentum, eps):
        N, H, W_, Cin = x.shape
        Cout, KH, KW, wcin = w.shape
        stem = Cin == 4 and wcin == 3
        OH, OW = (H + 2 * pad - KH) // stride + 1, (W_ + 2 * pad - KW) // stride + 1
        wb = w.to(BF16)
        if stem:
            wb = torch.nn.functional.pad(wb, (0, 1))
        wb = wb.contiguous()
        y = torch.empty(N, OH, OW, Cout, dtype=BF16, device=x.device)
        C = _C()
        nblk = C.conv_gemm_fwd_blocks(x, y, KH, KW, stride, pad)
        stats = torch.empty(nblk, 2, Cout, device=x.device) if training else None
        C.conv_gemm_fwd(x, wb, None, y, KH, KW, stride, pad, False, stats)
        P = N * OH * OW
        if training:
            mean = torch.empty(Cout, device=x.device)
            invstd = torch.empty(Cout, device=x.device)
            C.bn_finalize(stats, nblk, Cout, float(P), eps, momentum, running_mean, running_var,
                          mean, invstd)
        else:
            mean = running_mean.float().contiguous()
            invstd = torch.rsqrt(running_var.float() + eps).contiguous()
        out = torch.empty_like(y)
        C.bn_apply(y, mean, invstd, gamma.contiguous(), beta.contiguous(),
                   res.contiguous() if res is not None else None, bool(relu), out)
        ctx.save_for_backward(x, w, y, out, mean, invstd, gamma)
        ctx.cfg = (stride, pad, bool(relu), res is not None, stem, P)
        return out

    @staticmethod
    def backward(ctx, dout):
        x, w, y, out, mean, invstd, gamma = ctx.saved_tensors
        stride, pad, relu, has_res, stem, P = ctx.cfg
        C = _C()
        dout = dout.to(BF16).contiguous()
        Cout, KH, KW, wcin = w.shape
        rows = 256
        nb = C.bn_bwd_blocks(P, rows)
        slab = torch.empty(nb, 2 * Cout, device=dout.device)
        C.bn_bwd_reduce(dout, out if relu else None, y, mean, invstd, slab, rows)
        sums = torch.empty(2 * Cout, device=dout.device)
        C.grad_reduce([(slab, 2 * Cout, 0, 2 * Cout, nb, sums, 1.0)])
        dy = torch.empty_like(y)
        dres = torch.empty_like(y) if has_res else None
        C.bn_bwd_apply(dout, out if relu else None, y, mean, invstd, gamma.contiguous(), sums,
                       float(P), dy, dres)
        dgamma, dbeta = sums[Cout:].clone(), sums[:Cout].clone()
        dx = None
        if ctx.needs_input_grad[0] and not stem:
            wt = torch.empty(w.numel(), dtype=BF16, device=w.device)
            C.transpose_w(w.contiguous(), wt)
            dx = torch.empty_like(x)
            C.conv_gemm_dgrad(dy, wt, None, dx, KH, KW, stride, pad)
        gx = Cout // 64
        gy = (KH * KW + 15) // 16 if stem else KH * KW * (x.shape[3] // 64)
        ppc = _wgrad_ppc(P, gx, gy)
        chunks = C.conv_gemm_wgrad_chunks(x, dy, KH, KW, stride, pad, ppc)
        cin = x.shape[3]
        row = Cout * KH * KW * cin
        wslab = torch.empty(chunks, row, device=dout.device)
        C.conv_gemm_wgrad(dy, x, wslab, KH, KW, stride, pad, ppc)
        dw = torch.empty(row, device=dout.device)
        C.grad_reduce([(wslab, row, 0, row, chunks, dw, 1.0)])
        dw = dw.view(Cout, KH, KW, cin)
        if stem:
            dw = dw[..., :wcin].contiguous()
        return dx, dw, dgamma, dbeta, None, None, dres, None, None, None, None, None, None


class _MaxPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        N, H, W, Cc = x.shape
        OH, OW = (H - 1) // 2 + 1, (W - 1) // 2 + 1
        y = torch.empty(N, OH, OW, Cc, dtype=BF16, device=x.device)
        am = torch.empty(N, OH, OW, Cc, dtype=torch.uint8, device=x.device)
        _C().maxpool_fwd(x.contiguous(), y, am)
        ctx.save_for_backward(am)
        ctx.shape = x.shape
        return y

    @staticmethod
    def backward(ctx, dy):
        (am,) = ctx.saved_tensors
        dx = torch.empty(ctx.shape, dtype=BF16, device=dy.device)
        _C().maxpool_bwd(dy.to(BF16).contiguous(), am, dx)
        return dx


class _AvgPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        N, H, W, Cc = x.shape
        y = torch.empty(N, Cc, device=x.device)
        _C().avgpool_fwd(x.contiguous(), y)
        ctx.shape = x.shape
        return y

    @staticmethod
    def backward(ctx, dy):
        dx = torch.empty(ctx.shape, dtype=BF16, device=dy.device)
        _C().avgpool_bwd(dy.float().contiguous(), dx)
        return dx


class _LinearHead(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        B, K = x.shape
        N = w.shape[0]
        out = torch.empty(B, N, device=x.device)
        x = x.float().contiguous()
        w = w.contiguous()
        _C().sgemm(B, N, K, x, K, 1, w, 1, K, out, b.contiguous() if b is not None else None, 1.0)
        ctx.save_for_backward(x, w)
        ctx.has_bias = b is not None
        return out

    @staticmethod
    def backward(ctx, dl):
        x, w = ctx.saved_tensors
        B, K = x.shape
        N = w.shape[0]
        dl = dl.float().contiguous()
        dx = torch.empty(B, K, device=dl.device)
        _C().sgemm(B, K, N, dl, N, 1, w, K, 1, dx, None, 1.0)
        dw = torch.empty(N, K, device=dl.device)
        _C().sgemm(N, K, B, dl, 1, N, x, K, 1, dw, None, 1.0)
        db = dl.sum(0) if ctx.has_bias else None
        return dx, dw, db


def conv_bn_act(x, conv, bn, res=None, relu=True):
    training = bn.training
    if training and bn.track_running_stats:
        bn.num_batches_tracked.add_(1)
    momentum = bn.momentum if bn.momentum is not None else 0.1
    return _ConvBNAct.apply(x, conv.weight, bn.weight, bn.bias, bn.running_mean, bn.running_var,
                            res, conv.stride, conv.padding, relu, training, momentum, bn.eps)


def maxpool3x3s2(x):
    return _MaxPool.apply(x)


def global_avgpool(x):
    return _AvgPool.apply(x)


def linear_head(x, w, b):
    return _LinearHead.apply(x, w, b)
