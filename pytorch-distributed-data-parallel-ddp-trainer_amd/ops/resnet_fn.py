"""HIP autograd Functions for ResNet-style networks (NHWC bf16 activations).

==================  ================================================  ===========================================
Function            forward kernels                                   backward kernels
==================  ================================================  ===========================================
conv_bn_act         conv_gemm_fwd (+ BN sum/sumsq epilogue, or        bn_bwd (strip reduce -> dgamma/dbeta,
                    split-K partials -> splitk_reduce + stats),       apply), conv_gemm_dgrad (OHWI weight read
                    bn_finalize (running stats, batches tracked),     transposed in LDS), conv_gemm_wgrad (->
                    bn_apply (+ residual add + ReLU)                  grad, or slabs -> grad_reduce)
maxpool3x3s2        maxpool_fwd (argmax saved)                        maxpool_bwd (deterministic gather)
global_avgpool      avgpool_fwd                                       avgpool_bwd
linear_head         sgemm (in-tree fp32 GEMM, + bias)                 sgemm x3 (dx; dW and db accumulated in place)
==================  ================================================  ===========================================

Residual joins: a block's input x feeds its conv branch and its residual branch, so
autograd would add the two gradients with a separate bf16 add kernel.  Instead the
residual branch (``stash=``) parks its gradient in a :class:`GradStash` hung on x's
producer node, returns none, and the producer's backward (BatchNorm backward or the
maxpool backward) sums it into its upstream gradient while loading it - bitwise the same
bf16 sum, one kernel and one full pass fewer per block.

Weights: the MFMA operand is the model's flat bf16 parameter copy (``FlatSpace.bf16_params``,
refreshed by FusedSGD inside its update kernel) when the model is flattened (DDP /
FusedSGD), else a per-call conversion.  The stem's 3 input channels are zero-padded to 4
so its K-steps pack 8 taps x 4 channels.

Gradients: weight / BN-affine / fc gradients are accumulated straight into ``param.grad``
by the reducing kernel when allowed (:mod:`.direct_grad`), otherwise returned.
"""
from __future__ import annotations

import os

import torch

from .. import native
from . import direct_grad

BF16 = torch.bfloat16
# (Round 3 measured two BatchNorm launch-count reductions - the statistics finalised inside
# the stats-producing conv launch, and a one-launch BatchNorm backward - both slower on
# MI355X: 13.7k vs 14.2k img/s, profiles/r3_bn_fusion; removed in round 5.)
# BatchNorm backward of a ReLU without a residual add: the mask recomputed from the BN input
# (no read of the saved output in either pass); DDP_AMD_BN_MASK_FROM_Y=0 reads the output
MASK_FROM_Y = os.environ.get("DDP_AMD_BN_MASK_FROM_Y", "1") != "0"
# BatchNorm + ReLU without a residual add applied by the consumer's loads (no bn_apply
# pass): the stem's by the maxpool, each block's bn1 by conv2's halo forward and halo
# weight gradient; DDP_AMD_DEFER_BN=0 materialises them.  Needs MASK_FROM_Y (the output is
# never stored).
DEFER_BN = os.environ.get("DDP_AMD_DEFER_BN", "1") != "0" and MASK_FROM_Y
# (Weight gradients on a side stream - graph branches do overlap here, scripts/
# graph_branch_probe.py - measured 5 % slower over 1000 steps: the side-stream wgrad
# kernels share the CUs with the critical chain's own; profiles/r4_resnet/halo_pipe.)


def _C():
    return native.require()


def to_nhwc4(x: torch.Tensor) -> torch.Tensor:
    """NCHW float image batch -> NHWC bf16 with channels zero-padded to 4 (stem input)."""
    n, c, h, w = x.shape
    out = torch.zeros(n, h, w, 4, dtype=BF16, device=x.device)
    out[..., :c] = x.permute(0, 2, 3, 1)
    return out


class GradStash:
    """A second upstream gradient of a tensor, handed from one consumer's backward to the
    tensor producer's backward (see the module docstring)."""

    def __init__(self):
        self.grad = None

    def put(self, g):
        if g is None:
            return
        self.grad = g if self.grad is None else self.grad + g  # (never twice in a ResNet block)

    def take(self):
        g, self.grad = self.grad, None
        return g


def attach_stash(x: torch.Tensor):
    """A GradStash on x's producer node (its ctx in backward), or None when x has no
    producer that can consume one (then the residual branch returns its gradient)."""
    fn = x.grad_fn
    if fn is None or not isinstance(fn, (_ConvBNAct._backward_cls, _MaxPool._backward_cls)):
        return None
    st = getattr(fn, "_ddp_amd_stash", None)
    if st is None:
        st = GradStash()
        fn._ddp_amd_stash = st
    return st


def _take_stash(ctx):
    st = getattr(ctx, "_ddp_amd_stash", None)
    g = st.take() if st is not None else None
    return g.to(BF16).contiguous() if g is not None else None


def _weight_bf16(w: torch.Tensor) -> torch.Tensor:
    fs = getattr(w, "_ddp_amd_fs", None)
    v = fs.bf16_view(w) if fs is not None else None
    return v if v is not None else w.detach().to(BF16).contiguous()


class _ConvBNAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, gamma, beta, running_mean, running_var, nbt, res, stride, pad, relu,
                training, momentum, eps, stash=None, defer=False):
        N, H, W_, Cin = x.shape
        Cout, KH, KW, wcin = w.shape
        stem = Cin == 4 and wcin == 3
        OH, OW = (H + 2 * pad - KH) // stride + 1, (W_ + 2 * pad - KW) // stride + 1
        wb = _weight_bf16(w)
        wk = wb
        if stem:  # the padded copy FusedSGD keeps, else a per-call pad
            fs = getattr(w, "_ddp_amd_fs", None)
            wk = fs.bf16_pad4_view(w) if fs is not None else None
            if wk is None:
                wk = torch.nn.functional.pad(wb, (0, 1))
        y = torch.empty(N, OH, OW, Cout, dtype=BF16, device=x.device)
        C = _C()
        P = N * OH * OW
        _, _, splits, rows, _, halo = C.conv_gemm_plan(x, y, KH, KW, stride, pad)
        # x may be the producer's deferred BatchNorm + ReLU (raw conv output + affine): the
        # halo forward and the halo weight gradient apply it while staging; any other plan
        # gets the activation materialised here
        xbn = getattr(x, "_ddp_amd_bn", None)
        if xbn is not None:
            ppc = C.conv_gemm_wgrad_ppc(x, y, KH, KW, stride, pad)
            if not (halo == 1 and C.conv_gemm_wgrad_uses_halo(x, y, KH, KW, stride, pad, ppc)):
                xm = torch.empty_like(x)
                C.bn_apply(x, xbn[0], xbn[1], xbn[2], xbn[3], None, True, xm)
                x, xbn = xm, None
        part = torch.empty(splits * P * Cout, device=x.device) if splits > 1 else None
        stats = torch.empty(rows, 2, Cout, device=x.device) if training else None
        if training:
            mean = torch.empty(Cout, device=x.device)
            invstd = torch.empty(Cout, device=x.device)
        C.conv_gemm_fwd(x, wk, None, y, KH, KW, stride, pad, False, stats, part, bn=xbn)
        if training:
            ws = torch.empty(C.bn_finalize_groups(rows), 2, Cout, device=x.device)
            C.bn_finalize(stats, rows, Cout, float(P), eps, momentum, running_mean, running_var,
                          mean, invstd, nbt, ws)
        else:
            mean = running_mean.float().contiguous()
            invstd = torch.rsqrt(running_var.float() + eps).contiguous()
        if defer:
            # the consumer applies BN + ReLU while loading (BnAffine); the returned tensor
            # holds the RAW conv output, tagged with the affine, and stands for relu(bn(y))
            # in autograd (its gradient is d loss / d relu(bn(y)), as without deferral)
            assert relu and res is None, "deferred BatchNorm: ReLU, no residual add"
            out = y
            out._ddp_amd_bn = [mean, invstd, gamma.detach(), beta.detach()]
        else:
            out = torch.empty_like(y)
            C.bn_apply(y, mean, invstd, gamma.detach(), beta.detach(),
                       res.contiguous() if res is not None else None, bool(relu), out)
        # the backward's ReLU mask: without a residual add it is recomputed from y (bitwise
        # the sign of `out`, resnet_ops.hip bn_mask8), so `out` is kept only for a join
        keep_out = bool(relu) and (res is not None or not MASK_FROM_Y)
        ctx.save_for_backward(x, wb, y, out if keep_out else None, mean, invstd)
        ctx.params = (w, gamma, beta)
        ctx.xbn = xbn
        ctx.cfg = (stride, pad, bool(relu), res is not None, stem, P)
        # stash: this Function is the residual branch of a block; its gradient w.r.t. the
        # block input (res's for a join, x's for a downsample conv) goes to the stash
        ctx.stash = stash
        return out

    @staticmethod
    def backward(ctx, dout):
        x, wb, y, out, mean, invstd = ctx.saved_tensors
        w, gamma, beta = ctx.params
        stride, pad, relu, has_res, stem, P = ctx.cfg
        C = _C()
        dout = dout.to(BF16).contiguous()
        Cout, KH, KW, wcin = w.shape
        dev = dout.device
        # BatchNorm backward; dgamma / dbeta straight into the parameter gradients if allowed
        gg, gb = direct_grad.grad_dst(gamma), direct_grad.grad_dst(beta)
        direct_bn = gg is not None and gb is not None
        acc_bn = False
        if direct_bn:
            dgamma, dbeta = gg, gb
            ag, ab = direct_grad.accumulate(gamma), direct_grad.accumulate(beta)
            if ag != ab:  # (one of the pair fresh: clear it, then both add)
                (dbeta if ag else dgamma).zero_()
            acc_bn = ag or ab
        else:
            dgamma, dbeta = torch.empty(Cout, device=dev), torch.empty(Cout, device=dev)
        ws = torch.empty(C.bn_bwd_rows(P, Cout), 2, Cout, device=dev)
        sums = torch.empty(2 * Cout, device=dev)
        dy = torch.empty_like(y)
        dres = torch.empty_like(y) if has_res else None
        mask_beta = beta.detach() if (relu and out is None) else None
        C.bn_bwd(dout, out if relu else None, y, mean, invstd, gamma.detach(), float(P), ws, sums,
                 dgamma, dbeta, acc_bn, dy, dres, _take_stash(ctx), mask_beta)
        # data gradient (the stem's input is the image: none)
        dx = None
        if ctx.needs_input_grad[0] and not stem:
            dx = torch.empty_like(x)
            _, _, splits, _, _, _ = C.conv_gemm_plan(x, dout, KH, KW, stride, pad, True)
            part = torch.empty(splits * x.numel(), device=dev) if splits > 1 else None
            C.conv_gemm_dgrad(dy, wb, None, dx, KH, KW, stride, pad, part)
        # weight gradient
        gw = direct_grad.grad_dst(w)
        acc_w = gw is not None and direct_grad.accumulate(w)
        ppc = C.conv_gemm_wgrad_ppc(x, dy, KH, KW, stride, pad)
        chunks = C.conv_gemm_wgrad_chunks(x, dy, KH, KW, stride, pad, ppc)
        row = w.numel()
        dw = gw if gw is not None else torch.empty(w.shape, device=dev)
        if chunks == 1:
            C.conv_gemm_wgrad(dy, x, dw, KH, KW, stride, pad, ppc, acc_w, bn=ctx.xbn)
        else:
            slab = torch.empty(chunks, row, device=dev)
            C.conv_gemm_wgrad(dy, x, slab, KH, KW, stride, pad, ppc, False, bn=ctx.xbn)
            C.grad_reduce([(slab, row, 0, row, chunks, dw.view(-1), 1.0, acc_w)])
        rw = None if gw is not None else dw
        rg, rb = (None, None) if direct_bn else (dgamma, dbeta)
        if ctx.stash is not None:  # residual branch: hand the block-input gradient over
            if has_res:
                ctx.stash.put(dres)
                dres = None
            else:
                ctx.stash.put(dx)
                dx = None
        return dx, rw, rg, rb, None, None, None, dres, None, None, None, None, None, None, None, None


class _MaxPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        N, H, W, Cc = x.shape
        OH, OW = (H - 1) // 2 + 1, (W - 1) // 2 + 1
        y = torch.empty(N, OH, OW, Cc, dtype=BF16, device=x.device)
        am = torch.empty(N, OH, OW, Cc, dtype=torch.uint8, device=x.device)
        # a deferred BatchNorm + ReLU of the producer (conv_bn_act(defer=True)) is applied here
        _C().maxpool_fwd(x.contiguous(), y, am, getattr(x, "_ddp_amd_bn", None))
        ctx.save_for_backward(am)
        ctx.shape = x.shape
        return y

    @staticmethod
    def backward(ctx, dy):
        (am,) = ctx.saved_tensors
        dx = torch.empty(ctx.shape, dtype=BF16, device=dy.device)
        _C().maxpool_bwd(dy.to(BF16).contiguous(), am, dx, _take_stash(ctx))
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


_ONES: dict = {}


def _ones(n: int, device) -> torch.Tensor:
    """A persistent all-ones fp32 vector (the bias gradient's 1^T operand): a fresh
    ``torch.ones`` was a fill kernel inside every captured ResNet step (profiles/r6_resnet)."""
    key = (n, str(device))
    t = _ONES.get(key)
    if t is None:
        t = _ONES[key] = torch.ones(n, device=device)
    return t


class _LinearHead(torch.autograd.Function):
    """fp32 classifier head ([B,512] x [512,classes]) on the in-tree GEMM (``sgemm``): the
    forward with the bias folded in; the backward as dx = dl.W, dW += dl^T.x and
    db += 1^T.dl, the last two accumulated straight into the flat gradient views."""

    @staticmethod
    def forward(ctx, x, w, b):
        x = x.float().contiguous()
        B, K = x.shape
        N = w.shape[0]
        out = torch.empty(B, N, device=x.device)
        wd = w.detach()
        _C().sgemm(B, N, K, x, K, 1, wd, 1, K, out, b.detach() if b is not None else None, 1.0)
        ctx.save_for_backward(x)
        ctx.params = (w, b)
        return out

    @staticmethod
    def backward(ctx, dl):
        (x,) = ctx.saved_tensors
        w, b = ctx.params
        C = _C()
        dl = dl.float().contiguous()
        B, K = x.shape
        N = w.shape[0]
        wd = w.detach()
        dx = torch.empty(B, K, device=dl.device)
        C.sgemm(B, K, N, dl, N, 1, wd, K, 1, dx, None, 1.0)                    # dl . W
        gw = direct_grad.grad_dst(w)
        rw = None
        if gw is not None:
            C.sgemm(N, K, B, dl, 1, N, x, K, 1, gw, None, 1.0, direct_grad.accumulate(w))  # dW (+)= dl^T . x
        else:
            rw = torch.empty(N, K, device=dl.device)
            C.sgemm(N, K, B, dl, 1, N, x, K, 1, rw, None, 1.0)
        rb = None
        if b is not None:
            ones = _ones(B, dl.device)
            gb = direct_grad.grad_dst(b)
            if gb is not None:
                C.sgemm(1, N, B, ones, 0, 1, dl, N, 1, gb, None, 1.0, direct_grad.accumulate(b))  # db (+)= 1^T . dl
            else:
                rb = torch.empty(N, device=dl.device)
                C.sgemm(1, N, B, ones, 0, 1, dl, N, 1, rb, None, 1.0)
        return dx, rw, rb


def conv_bn_act(x, conv, bn, res=None, relu=True, stash=None, defer=False):
    """conv -> BatchNorm -> (+ res) -> (ReLU).  defer=True (ReLU, no residual): the BN + ReLU
    is left to the consumer's loads (maxpool3x3s2, or conv_bn_act: halo plans apply it while
    staging, others materialise it); the result must only be passed to such a consumer."""
    training = bn.training
    nbt = bn.num_batches_tracked if (training and bn.track_running_stats) else None
    momentum = bn.momentum if bn.momentum is not None else 0.1
    return _ConvBNAct.apply(x, conv.weight, bn.weight, bn.bias, bn.running_mean, bn.running_var,
                            nbt, res, conv.stride, conv.padding, relu, training, momentum, bn.eps, stash,
                            bool(defer) and DEFER_BN)


def maxpool3x3s2(x):
    return _MaxPool.apply(x)


def global_avgpool(x):
    return _AvgPool.apply(x)


def linear_head(x, w, b):
    return _LinearHead.apply(x, w, b)
