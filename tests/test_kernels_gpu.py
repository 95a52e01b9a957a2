"""Numerics of every gfx950 HIP kernel against a plain PyTorch fp32 reference of the same op.

Inputs are bf16-representable (the kernels' operand precision), the reference runs
in fp32 on those exact values, and outputs are compared at bf16 output precision.
Batch sizes cover the ragged last batches of the reference's epochs (SURVEY §3.4:
12, 16, 24, 48 besides 32/64) and B=1.
"""
import pytest
import torch

from ddp_amd.ops import reference as R

pytestmark = pytest.mark.gpu
dev = "cuda"
BF = torch.bfloat16


def rnd(*shape, scale=1.0, seed=0, relu=False):
    g = torch.Generator().manual_seed(seed)
    t = torch.randn(*shape, generator=g) * scale
    if relu:
        t = torch.relu(t)
    return t.to(BF).to(dev)


def close(a, b, rtol=2e-2, atol=2e-2):
    torch.testing.assert_close(a.float().cpu(), b.float().cpu(), rtol=rtol, atol=atol)


def relclose(a, b, tol=1e-2):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).norm() / b.norm().clamp_min(1e-12)
    assert err < tol, f"relative error {err:.3e}"


@pytest.mark.parametrize("B", [1, 12, 32])
def test_conv1_fwd_float_and_u8(C, B):
    H = W = 28
    g = torch.Generator().manual_seed(1)
    w = (torch.randn(32, 3, 3, 1, generator=g) * 0.3).to(dev)
    b = (torch.randn(32, generator=g) * 0.1).to(dev)
    x = torch.rand(B, H * W, generator=g).to(dev)
    y = torch.empty(B, H, W, 32, dtype=BF, device=dev)
    C.conv1_fwd(x, None, None, 0, 0, w, b, y, B, H, W)
    ref = R.conv1_relu(x.view(B, H, W), w, b)
    close(y, R.bf16r(ref), rtol=1e-2, atol=1e-2)
    # u8 dataset + index gather with ToTensor's /255 fused
    N = 100
    data = torch.randint(0, 256, (N, H, W), generator=g, dtype=torch.uint8).to(dev)
    idx = torch.randperm(N, generator=g)[: B + 5].to(torch.int32).to(dev)
    y2 = torch.empty_like(y)
    C.conv1_fwd(data, idx, None, 0, 5, w, b, y2, B, H, W)
    xs = data[idx[5:5 + B].long()].float() / 255.0
    close(y2, R.bf16r(R.conv1_relu(xs, w, b)), rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("B,pxt", [(1, 1), (12, 2), (32, 2), (24, 1)])
def test_conv3x3_fwd(C, B, pxt):
    H = W = 28
    x = rnd(B, H, W, 32, relu=True, seed=2)
    w = rnd(64, 3, 3, 32, scale=0.1, seed=3)
    b = (torch.randn(64) * 0.1).to(dev)
    y = torch.empty(B, H, W, 64, dtype=BF, device=dev)
    C.conv3x3_fwd(x, w, b, y, True, None, None, 0, pxt)
    ref = R.conv3x3(x.float(), w.float(), b, relu=True)
    close(y, ref)


@pytest.mark.parametrize("B", [1, 16, 32])
def test_conv3x3_fwd_fused_fc(C, B):
    H = W = 28
    x = rnd(B, H, W, 32, relu=True, seed=4)
    w = rnd(64, 3, 3, 32, scale=0.1, seed=5)
    b = (torch.randn(64) * 0.1).to(dev)
    wfc = rnd(10, H * W, 64, scale=0.01, seed=6)
    bfc = (torch.randn(10) * 0.1).to(dev)
    y = torch.empty(B, H, W, 64, dtype=BF, device=dev)
    nblk = C.conv3x3_dgrad_blocks(B, H, W, 2)  # conv blocks of 128 pixels
    part = torch.full((nblk, 2, 10), float("nan"), device=dev)
    from ddp_amd.ops.functional import fc_weight_frag, fold_block_partials

    C.conv3x3_fwd(x, w, b, y, True, fc_weight_frag(wfc, H * W, 64), part, 10, 2)
    logits = fold_block_partials(part, B, H * W, 128) + bfc
    ref = R.fc_nhwc(y.float(), wfc.float(), bfc)  # the fc of exactly the stored bf16 activation
    close(logits, ref, rtol=1e-3, atol=1e-3)
    # engine cross-entropy over those [blocks][2][10] partials (+ fc bias grad / mean loss in fc_bwd)
    labels = torch.randint(0, 10, (B,)).to(torch.int32).to(dev)
    dl = torch.empty(B, 10, device=dev)
    rows = torch.empty(B, device=dev)
    C.xent_rows(part, H * W, 128, bfc, labels, None, dl, rows, 1.0 / B)
    rl, rd = R.cross_entropy(ref, labels.long())
    close(dl, rd, rtol=1e-4, atol=1e-6)
    close(rows.mean(), rl, rtol=1e-5, atol=1e-5)
    dx = torch.empty_like(y)
    dw = torch.empty(10, 28 * 28, 64, device=dev)
    db = torch.empty(10, device=dev)
    loss = torch.zeros(3, device=dev)
    C.fc_bwd(dl, y, wfc, dx, dw, 0.5, True, db, rows, loss)
    close(db, 0.5 * rd.sum(0), rtol=1e-5, atol=1e-7)
    close(loss[0], rl, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("mask_dy,mask_x", [(True, False), (False, True), (True, True), (False, False)])
def test_conv3x3_dgrad(C, mask_dy, mask_x):
    B, H, W = 12, 28, 28
    dy = rnd(B, H, W, 64, scale=0.5, seed=7)
    yact = rnd(B, H, W, 64, seed=8)
    xact = rnd(B, H, W, 32, seed=9)
    w = rnd(64, 3, 3, 32, scale=0.1, seed=10)
    wt = w.view(64, 9, 32).permute(1, 2, 0).contiguous()
    dx = torch.empty(B, H, W, 32, dtype=BF, device=dev)
    C.conv3x3_dgrad(dy, yact if mask_dy else None, wt, xact if mask_x else None, dx, 2)
    g = dy.float() * (yact.float() > 0) if mask_dy else dy.float()
    ref = R.conv3x3_dgrad(g, w.float())
    if mask_x:
        ref = ref * (xact.float() > 0)
    close(dx, ref)


@pytest.mark.parametrize("B,Rrows", [(1, 14), (12, 7), (32, 14), (16, 4)])
def test_conv3x3_wgrad(C, B, Rrows):
    H = W = 28
    dy = rnd(B, H, W, 64, scale=0.5, seed=11)
    yact = rnd(B, H, W, 64, seed=12)
    x = rnd(B, H, W, 32, relu=True, seed=13)
    nblk = C.conv3x3_wgrad_blocks(B, H, Rrows)
    row = 64 * 9 * 32 + 64
    slab = torch.full((nblk, row), float("nan"), device=dev)
    C.conv3x3_wgrad(dy, yact, x, slab, Rrows)
    gw = torch.empty(64 * 9 * 32, device=dev)
    gb = torch.empty(64, device=dev)
    C.grad_reduce([(slab, row, 0, 64 * 9 * 32, nblk, gw, 1.0), (slab, row, 64 * 9 * 32, 64, nblk, gb, 1.0)])
    g = dy.float() * (yact.float() > 0)
    rw, rb = R.conv3x3_wgrad(g, x.float())
    relclose(gw.view(64, 3, 3, 32), rw, 2e-3)
    relclose(gb, rb, 2e-3)
    # bitwise determinism (fixed-order split-K, no atomics)
    gw2 = torch.empty_like(gw)
    slab2 = torch.empty_like(slab)
    C.conv3x3_wgrad(dy, yact, x, slab2, Rrows)
    C.grad_reduce([(slab2, row, 0, 64 * 9 * 32, nblk, gw2, 1.0)])
    assert torch.equal(gw, gw2)


@pytest.mark.parametrize("B", [1, 24])
def test_conv1_wgrad(C, B):
    H = W = 28
    g0 = torch.Generator().manual_seed(14)
    x = torch.rand(B, H * W, generator=g0).to(dev)
    dy = rnd(B, H, W, 32, scale=0.5, seed=15)
    yact = rnd(B, H, W, 32, seed=16)
    chunk = 256
    nblk = C.conv1_wgrad_blocks(B, H, W, chunk)
    slab = torch.empty(nblk, 320, device=dev)
    C.conv1_wgrad(x, None, None, 0, 0, dy, yact, slab, B, H, W, 32, chunk)
    gw = torch.empty(288, device=dev)
    gb = torch.empty(32, device=dev)
    C.grad_reduce([(slab, 320, 0, 288, nblk, gw, 1.0), (slab, 320, 288, 32, nblk, gb, 1.0)])
    rw, rb = R.conv1_wgrad(dy.float() * (yact.float() > 0), x.view(B, H, W))
    relclose(gw.view(32, 3, 3, 1), rw, 2e-3)
    relclose(gb, rb, 2e-3)


def test_conv3x3_dgrad_fused_conv1_wgrad(C):
    B, H, W = 12, 28, 28
    g0 = torch.Generator().manual_seed(17)
    N = 64
    data = torch.randint(0, 256, (N, H, W), generator=g0, dtype=torch.uint8).to(dev)
    idx = torch.randperm(N, generator=g0)[:B].to(torch.int32).to(dev)
    dy = rnd(B, H, W, 64, scale=0.5, seed=18)
    a1 = rnd(B, H, W, 32, seed=19)
    w = rnd(64, 3, 3, 32, scale=0.1, seed=20)
    wt = w.view(64, 9, 32).permute(1, 2, 0).contiguous()
    dz1 = torch.empty(B, H, W, 32, dtype=BF, device=dev)
    nblk = C.conv3x3_dgrad_blocks(B, H, W, 2)
    slab = torch.empty(nblk, 320, device=dev)
    C.conv3x3_dgrad_fused_w1(dy, wt, a1, dz1, data, idx, None, 0, 0, slab, 2)
    ref_dz1 = R.conv3x3_dgrad(dy.float(), w.float()) * (a1.float() > 0)
    close(dz1, ref_dz1)
    gw = torch.empty(288, device=dev)
    gb = torch.empty(32, device=dev)
    C.grad_reduce([(slab, 320, 0, 288, nblk, gw, 1.0), (slab, 320, 288, 32, nblk, gb, 1.0)])
    x = data[idx.long()].float() / 255.0
    rw, rb = R.conv1_wgrad(dz1.float(), x)  # from the stored bf16 dZ1, as the kernel does
    relclose(gw.view(32, 3, 3, 1), rw, 2e-3)
    relclose(gb, rb, 2e-3)


@pytest.mark.parametrize("B", [1, 32])
def test_fc_fwd_bwd(C, B):
    H = W = 28
    x = rnd(B, H, W, 64, relu=True, seed=21)
    wfc = rnd(10, H * W, 64, scale=0.01, seed=22)
    bfc = (torch.randn(10) * 0.1).to(dev)
    part = torch.empty(B, 49, 10, device=dev)
    C.fc_partial(x, wfc, part)
    out = torch.empty(B, 10, device=dev)
    C.fc_reduce(part, bfc, out, B, 49, 10)
    close(out, R.fc_nhwc(x.float(), wfc.float(), bfc), rtol=1e-3, atol=1e-3)
    dl = (torch.randn(B, 10) * 0.1).to(dev)
    for mask in (True, False):
        dx = torch.empty_like(x)
        dw = torch.empty(10, H * W, 64, device=dev)
        C.fc_bwd(dl, x, wfc, dx, dw, 0.5, mask)
        rdx, rdw = R.fc_bwd(dl, x.float(), wfc.float(), mask=mask)
        close(dx, rdx, rtol=2e-2, atol=1e-3)
        close(dw, 0.5 * rdw, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("B,G,Ccls", [(32, 49, 10), (7, 1, 10), (16, 1, 1000)])
def test_xent(C, B, G, Ccls):
    g0 = torch.Generator().manual_seed(23)
    part = (torch.randn(B, G, Ccls, generator=g0) * 0.5).to(dev)
    bias = (torch.randn(Ccls, generator=g0) * 0.1).to(dev)
    labels = torch.randint(0, Ccls, (B,), generator=g0).to(dev)
    dl = torch.empty(B, Ccls, device=dev)
    loss = torch.empty(1, device=dev)
    db = torch.empty(Ccls, device=dev)
    logits = torch.empty(B, Ccls, device=dev)
    C.xent(part, G, bias, labels, logits, dl, loss, db, 1.0 / B, 0.25)
    ref_logits = part.sum(1) + bias
    rl, rd = R.cross_entropy(ref_logits, labels)
    close(logits, ref_logits, rtol=1e-5, atol=1e-5)
    close(loss, rl.reshape(1), rtol=1e-5, atol=1e-5)
    close(dl, rd, rtol=1e-4, atol=1e-6)
    close(db, 0.25 * rd.sum(0), rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("momentum,nesterov,wd", [(0.0, False, 0.0), (0.9, False, 1e-4), (0.9, True, 0.0)])
def test_sgd_matches_torch(C, momentum, nesterov, wd):
    n = 10_000
    g0 = torch.Generator().manual_seed(24)
    p0 = torch.randn(n, generator=g0)
    grads = [torch.randn(n, generator=g0) for _ in range(3)]
    ref = torch.nn.Parameter(p0.clone())
    opt = torch.optim.SGD([ref], lr=0.01, momentum=momentum, nesterov=nesterov, weight_decay=wd)
    p = p0.clone().to(dev)
    mb = torch.zeros(n, device=dev)
    shadow = torch.empty(100, dtype=BF, device=dev)
    for i, gr in enumerate(grads):
        ref.grad = gr.clone()
        opt.step()
        C.sgd(p, gr.to(dev), mb, 0.01, momentum, 0.0, wd, nesterov, False, i == 0, True,
              [(50, 100, shadow, 1, 0, 0, 0)])
    close(p, ref.detach(), rtol=1e-6, atol=1e-6)
    assert torch.equal(shadow.cpu(), p[50:150].to(BF).cpu())


def test_sgd_transposed_shadow(C):
    w = torch.randn(64 * 9 * 32, device=dev)
    g = torch.zeros_like(w)
    sh = torch.empty(64 * 9 * 32, dtype=BF, device=dev)
    C.sgd(w, g, None, 0.0, 0.0, 0.0, 0.0, False, False, False, False, [(0, w.numel(), sh, 2, 64, 9, 32)])
    ref = w.view(64, 9, 32).permute(1, 2, 0).contiguous().view(-1).to(BF)
    assert torch.equal(sh.cpu(), ref.cpu())


def test_sgd_fcfrag_shadow(C):
    from ddp_amd.ops.functional import fc_weight_frag

    w = torch.randn(10 * 784 * 64, device=dev)
    sh = torch.empty(w.numel(), dtype=BF, device=dev)
    C.sgd(w, torch.zeros_like(w), None, 0.0, 0.0, 0.0, 0.0, False, False, False, False,
          [(0, w.numel(), sh, 3, 784, 64, 0)])
    assert torch.equal(sh.cpu(), fc_weight_frag(w, 784, 64).view(-1).cpu())


def _native_params(model):
    return {"w1": model.net[0].weight.detach(), "b1": model.net[0].bias.detach(),
            "w2": model.net[2].weight.detach(), "b2": model.net[2].bias.detach(),
            "wfc": model.fl.weight.detach(), "bfc": model.fl.bias.detach()}


def test_simple_cnn_module_path_matches_references():
    """SimpleCNN on cuda (HIP autograd Functions) vs (a) a bf16-emulating fp32 model of the
    same rounding points (tight) and (b) the plain fp32 CPU model (bf16-level tolerance)."""
    from ddp_amd.models import SimpleCNN
    from ddp_amd.ops import CrossEntropyLoss

    torch.manual_seed(0)
    cpu = SimpleCNN()
    gpu = SimpleCNN().to(dev)
    gpu.load_state_dict(cpu.state_dict())
    g0 = torch.Generator().manual_seed(25)
    x = torch.rand(16, 1, 28, 28, generator=g0)
    y = torch.randint(0, 10, (16,), generator=g0)
    loss_c = torch.nn.functional.cross_entropy(cpu(x), y)
    loss_c.backward()
    loss_g = CrossEntropyLoss()(gpu(x.to(dev)), y.to(dev))
    loss_g.backward()
    assert abs(loss_g.item() - loss_c.item()) < 2e-2
    # bf16-justified bound: the bf16 rounding model itself (ops/reference.py
    # simple_cnn_step_bf16, float math) deviates from the exact step (simple_cnn_step_exact,
    # float64) by e_k per parameter (measured here: 4.8e-2 / 5.5e-2 on conv1 w / b, 3e-3 on
    # fc); the HIP path may deviate from the fp32 model by at most 1.25 e_k + 1e-3.
    # (The exact-fp32 path is held to 1e-4: tests/test_fp32_gpu.py.)
    pe = {k: v.detach().cpu() for k, v in _native_params(cpu).items()}
    _, g_b = R.simple_cnn_step_bf16(pe, x.view(16, 28, 28), y)
    _, g_x = R.simple_cnn_step_exact(pe, x.view(16, 28, 28), y)
    key = {"net.0.weight": "w1", "net.0.bias": "b1", "net.2.weight": "w2", "net.2.bias": "b2",
           "fl.weight": "wfc", "fl.bias": "bfc"}
    for (n, pc), (_, pg) in zip(cpu.named_parameters(), gpu.named_parameters()):
        k = key[n]
        e_k = ((g_b[k].double() - g_x[k]).norm() / g_x[k].norm()).item()
        relclose(pg.grad, pc.grad, 1.25 * e_k + 1e-3)
    p = {k: v.cpu() for k, v in _native_params(gpu).items()}
    loss_e, ge = R.simple_cnn_step_bf16(p, x.view(16, 28, 28), y)
    assert abs(loss_g.item() - loss_e.item()) < 1e-4
    grads = {"w1": gpu.net[0].weight.grad, "b1": gpu.net[0].bias.grad, "w2": gpu.net[2].weight.grad,
             "b2": gpu.net[2].bias.grad, "wfc": gpu.fl.weight.grad, "bfc": gpu.fl.bias.grad}
    for k in ge:
        relclose(grads[k], ge[k], 1e-2)
