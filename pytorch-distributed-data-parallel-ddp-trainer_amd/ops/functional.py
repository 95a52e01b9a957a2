"""Autograd Functions over the gfx950 HIP kernels (the module path on MI355X).

Each Function wraps a fused kernel pair from ``csrc/kernels``:

===================  ==========================================  ==============================
op                   forward kernel                              backward kernels
===================  ==========================================  ==============================
conv1_relu           conv1_fwd (VALU, Cin=1, bias+ReLU fused)    conv1_wgrad (+ReLU mask) -> grad_reduce
conv3x3_relu         conv3x3_fwd (MFMA, bias+ReLU fused)         conv3x3_dgrad (+mask), conv3x3_wgrad -> grad_reduce
linear_nhwc          fc_partial + fc_reduce (split-K, fixed)     fc_bwd (dgrad+wgrad in one pass)
cross_entropy        xent (softmax-xent fwd+bwd fused)           scale of the saved dlogits
===================  ==========================================  ==============================

Activations are NHWC in the compute dtype: bf16 (default; fp32 masters converted to bf16
on the fly for the MFMA operands) or fp32 (``dtype=torch.float32``: exact-fp32 MFMA
``v_mfma_f32_16x16x4_f32`` conv2, fp32 fc, the reference's precision - the weights are
read as they are).
These functions require CUDA tensors and the native extension: there is no
silent PyTorch fallback on the GPU.
"""
from __future__ import annotations

import torch

from .. import native

BF16 = torch.bfloat16


def _C():
    return native.require()


def wgrad_rows(H: int, B: int, dtype=BF16) -> int:
    """Rows per wgrad block: the largest chunk that still gives >= 128 split-K blocks,
    capped at 7 rows (bf16) / 4 rows (fp32).

    Fewer, fatter blocks mean fewer fp32 slab rows to write and re-read, but the wgrad
    role shares the conv-backward launch with the data gradient and a fat block becomes
    its critical path.  Measured on MI355X (profiles/r2_perf/sweep.jsonl, 28x28x(32,64)):
    bf16 B=32: R=7 41.9 us/step vs R=14 51.5, R=4 43.3; B=64: R=7 62.8 vs R=14 72.9;
    fp32 B=32: R=4 83.4 vs R=7 92.3 (twice the LDS bytes per staged row).
    """
    for R in ((7, 4, 2, 1) if dtype == BF16 else (4, 2, 1)):
        if R <= H and B * ((H + R - 1) // R) >= 128:
            return R
    return 1


class _Conv1ReLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, dtype=BF16):
        B = x.shape[0]
        H, W = x.shape[-2], x.shape[-1]
        Cout = b.numel()
        xf = x.reshape(B, H * W).float().contiguous()
        y = torch.empty(B, H, W, Cout, dtype=dtype, device=x.device)
        _C().conv1_fwd(xf, None, None, 0, 0, w.contiguous(), b.contiguous(), y, B, H, W)
        ctx.save_for_backward(xf, y, w)
        ctx.dims = (B, H, W, Cout, tuple(x.shape))
        return y

    @staticmethod
    def backward(ctx, gy):
        xf, y, w = ctx.saved_tensors
        B, H, W, Cout, xshape = ctx.dims
        gy = gy.to(y.dtype).contiguous()
        chunk = 256
        nblk = _C().conv1_wgrad_blocks(B, H, W, chunk)
        slab = torch.empty(nblk, Cout * 10, dtype=torch.float32, device=gy.device)
        _C().conv1_wgrad(xf, None, None, 0, 0, gy, y, slab, B, H, W, Cout, chunk)
        gw = torch.empty(Cout * 9, dtype=torch.float32, device=gy.device)
        gb = torch.empty(Cout, dtype=torch.float32, device=gy.device)
        _C().grad_reduce([(slab, Cout * 10, 0, Cout * 9, nblk, gw, 1.0),
                          (slab, Cout * 10, Cout * 9, Cout, nblk, gb, 1.0)])
        gx = None
        if ctx.needs_input_grad[0]:  # rare (input images never require grad in training)
            dz = (gy.float() * (y.float() > 0)).permute(0, 3, 1, 2)
            gx = torch.nn.functional.conv_transpose2d(dz, w.permute(0, 3, 1, 2), padding=1)
            gx = gx.reshape(xshape)
        return gx, gw.view(Cout, 3, 3, 1), gb, None


class _Conv3x3ReLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, relu, dtype=BF16):
        B, H, W, Cin = x.shape
        Cout = w.shape[0]
        xb = x.to(dtype).contiguous()
        wb = w.to(dtype).contiguous()
        y = torch.empty(B, H, W, Cout, dtype=dtype, device=x.device)
        _C().conv3x3_fwd(xb, wb, b.contiguous(), y, bool(relu), None, None, 0, 2)
        ctx.save_for_backward(xb, wb, y)
        ctx.relu = bool(relu)
        return y

    @staticmethod
    def backward(ctx, gy):
        xb, wb, y = ctx.saved_tensors
        B, H, W, Cin = xb.shape
        Cout = wb.shape[0]
        gy = gy.to(xb.dtype).contiguous()
        yact = y if ctx.relu else None
        dx = None
        if ctx.needs_input_grad[0]:
            wt = wb.view(Cout, 9, Cin).permute(1, 2, 0).contiguous()  # [tap][ci][co]
            dx = torch.empty_like(xb)
            _C().conv3x3_dgrad(gy, yact, wt, None, dx, 2)
        R = wgrad_rows(H, B, xb.dtype)
        nblk = _C().conv3x3_wgrad_blocks(B, H, R)
        row = Cout * 9 * Cin + Cout
        slab = torch.empty(nblk, row, dtype=torch.float32, device=gy.device)
        _C().conv3x3_wgrad(gy, yact, xb, slab, R)
        gw = torch.empty(Cout * 9 * Cin, dtype=torch.float32, device=gy.device)
        gb = torch.empty(Cout, dtype=torch.float32, device=gy.device)
        _C().grad_reduce([(slab, row, 0, Cout * 9 * Cin, nblk, gw, 1.0),
                          (slab, row, Cout * 9 * Cin, Cout, nblk, gb, 1.0)])
        return dx, gw.view(Cout, 3, 3, Cin), gb, None, None


class _LinearNHWC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, dtype=BF16):
        B, H, W, C = x.shape
        NO = w.shape[0]
        xb = x.to(dtype).contiguous()
        wb = w.to(dtype).contiguous()
        G = (H * W) // 16
        part = torch.empty(B, G, NO, dtype=torch.float32, device=x.device)
        _C().fc_partial(xb, wb, part)
        out = torch.empty(B, NO, dtype=torch.float32, device=x.device)
        _C().fc_reduce(part, b.contiguous() if b is not None else None, out, B, G, NO)
        ctx.save_for_backward(xb, wb)
        ctx.has_bias = b is not None
        return out

    @staticmethod
    def backward(ctx, go):
        xb, wb = ctx.saved_tensors
        go = go.float().contiguous()
        dx = torch.empty_like(xb)
        dw = torch.empty(wb.shape, dtype=torch.float32, device=go.device)
        _C().fc_bwd(go, xb, wb, dx, dw, 1.0, False)
        db = go.sum(0) if ctx.has_bias else None
        return dx, dw, db, None


class _CrossEntropy(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels):
        B, C = logits.shape
        lg = logits.float().contiguous()
        dl = torch.empty_like(lg)
        loss = torch.empty(1, dtype=torch.float32, device=lg.device)
        _C().xent(lg, 1, None, labels.contiguous(), None, dl, loss, None, 1.0 / B, 0.0)
        ctx.save_for_backward(dl)
        return loss.reshape(())

    @staticmethod
    def backward(ctx, g):
        (dl,) = ctx.saved_tensors
        return dl * g, None


def conv1_relu(x, w, b, dtype=BF16):
    return _Conv1ReLU.apply(x, w, b, dtype)


def conv3x3_relu(x, w, b, relu=True, dtype=BF16):
    return _Conv3x3ReLU.apply(x, w, b, relu, dtype)


def linear_nhwc(x, w, b, dtype=BF16):
    return _LinearNHWC.apply(x, w, b, dtype)


def cross_entropy(logits, labels):
    return _CrossEntropy.apply(logits, labels)


def fc_weight_frag(w: torch.Tensor, hw: int, c: int, dtype=torch.bfloat16) -> torch.Tensor:
    """fc weight [out][H*W][C] (NHWC order) -> the MFMA-fragment order read by the fused
    FC epilogue of conv3x3_fwd (csrc SHADOW_BF16_FCFRAG / SHADOW_F32_FCFRAG):
    [out][hw/16][c/16][(c/4)%4][hw%16][c%4], bf16 (fp32 for the exact-fp32 forward)."""
    no = w.numel() // (hw * c)
    v = w.reshape(no, hw // 16, 16, c // 16, 4, 4)
    return v.permute(0, 1, 3, 4, 2, 5).contiguous().to(dtype)


def fold_block_partials(part: torch.Tensor, B: int, HW: int, CH: int) -> torch.Tensor:
    """Logits (without bias) from the fused conv2+fc epilogue's per-block partials.

    ``part`` is [blocks][2][NO]: block k covers pixels [k*CH, (k+1)*CH) of the flattened
    [B*HW] space; slot 0 belongs to the image of its first pixel, slot 1 to the next
    image (csrc/kernels/common.h xent_batch_block).  Reference/test helper."""
    nblk, _, NO = part.shape
    out = torch.zeros(B, NO, dtype=part.dtype, device=part.device)
    for k in range(nblk):
        n0 = (k * CH) // HW
        out[n0] += part[k, 0]
        if n0 + 1 < B and ((k + 1) * CH - 1) // HW > n0:
            out[n0 + 1] += part[k, 1]
    return out
