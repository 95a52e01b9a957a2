"""ResNet-18 kernels (conv_gemm, BatchNorm, pooling, head) vs plain PyTorch fp32 on MI355X."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
dev = "cuda"
BF = torch.bfloat16


def rnd(*shape, scale=1.0, seed=0, relu=False):
    g = torch.Generator().manual_seed(seed)
    t = torch.randn(*shape, generator=g) * scale
    return (torch.relu(t) if relu else t).to(BF).to(dev)


def relerr(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


CASES = [  # N, H, Cin, Cout, K, stride, pad
    (4, 14, 64, 64, 3, 1, 1),
    (4, 14, 64, 128, 3, 2, 1),
    (4, 14, 64, 128, 1, 2, 0),
    (2, 8, 256, 512, 3, 2, 1),
    (2, 7, 512, 512, 3, 1, 1),
]


@pytest.mark.parametrize("N,H,Cin,Cout,K,s,p", CASES)
def test_conv_gemm_fwd_dgrad_wgrad(C, N, H, Cin, Cout, K, s, p):
    OH = (H + 2 * p - K) // s + 1
    x = rnd(N, H, H, Cin, relu=True, seed=1)
    w = rnd(Cout, K, K, Cin, scale=0.05, seed=2)
    y = torch.empty(N, OH, OH, Cout, dtype=BF, device=dev)
    nblk = C.conv_gemm_fwd_blocks(x, y, K, K, s, p)
    stats = torch.empty(nblk, 2, Cout, device=dev)
    C.conv_gemm_fwd(x, w, None, y, K, K, s, p, False, stats)
    xr = x.float().permute(0, 3, 1, 2)
    wr = w.float().permute(0, 3, 1, 2)
    ref = F.conv2d(xr, wr, stride=s, padding=p).permute(0, 2, 3, 1)
    assert relerr(y, ref) < 1e-2
    yb = y.float()
    st = stats.sum(0)
    assert relerr(st[0], yb.sum((0, 1, 2))) < 1e-4
    assert relerr(st[1], (yb * yb).sum((0, 1, 2))) < 1e-4
    # data gradient
    dy = rnd(N, OH, OH, Cout, scale=0.5, seed=3)
    wt = torch.empty(w.numel(), dtype=BF, device=dev)
    C.transpose_w(w.float().contiguous(), wt)
    dx = torch.empty_like(x)
    C.conv_gemm_dgrad(dy, wt, None, dx, K, K, s, p)
    rdx = torch.nn.grad.conv2d_input(xr.shape, wr, dy.float().permute(0, 3, 1, 2), stride=s, padding=p)
    assert relerr(dx, rdx.permute(0, 2, 3, 1)) < 1e-2
    # weight gradient (split-K slabs + fixed-order reduce), bitwise reproducible
    P = N * OH * OH
    ppc = 64
    ch = C.conv_gemm_wgrad_chunks(x, dy, K, K, s, p, ppc)
    row = Cout * K * K * Cin
    slab = torch.empty(ch, row, device=dev)
    C.conv_gemm_wgrad(dy, x, slab, K, K, s, p, ppc)
    dw = torch.empty(row, device=dev)
    C.grad_reduce([(slab, row, 0, row, ch, dw, 1.0)])
    rdw = torch.nn.grad.conv2d_weight(xr, wr.shape, dy.float().permute(0, 3, 1, 2), stride=s, padding=p)
    assert relerr(dw.view(Cout, K, K, Cin), rdw.permute(0, 2, 3, 1)) < 2e-3


def test_stem_conv_7x7_s2():
    from ddp_amd import native
    from ddp_amd.ops.resnet_fn import to_nhwc4

    C = native.require()
    N, H = 2, 32
    img = torch.randn(N, 3, H, H, device=dev)
    x4 = to_nhwc4(img)
    w3 = torch.randn(64, 7, 7, 3) * 0.05
    w4 = F.pad(w3, (0, 1)).to(BF).to(dev).contiguous()
    OH = (H + 6 - 7) // 2 + 1
    y = torch.empty(N, OH, OH, 64, dtype=BF, device=dev)
    C.conv_gemm_fwd(x4, w4, None, y, 7, 7, 2, 3, False, None)
    ref = F.conv2d(x4[..., :3].float().permute(0, 3, 1, 2), w4[..., :3].float().permute(0, 3, 1, 2),
                   stride=2, padding=3).permute(0, 2, 3, 1)
    assert relerr(y, ref) < 1e-2
    dy = rnd(N, OH, OH, 64, seed=5)
    ppc = 64
    ch = C.conv_gemm_wgrad_chunks(x4, dy, 7, 7, 2, 3, ppc)
    slab = torch.empty(ch, 64 * 49 * 4, device=dev)
    C.conv_gemm_wgrad(dy, x4, slab, 7, 7, 2, 3, ppc)
    dw = torch.empty(64 * 49 * 4, device=dev)
    C.grad_reduce([(slab, 64 * 49 * 4, 0, 64 * 49 * 4, ch, dw, 1.0)])
    rdw = torch.nn.grad.conv2d_weight(x4[..., :3].float().permute(0, 3, 1, 2), (64, 3, 7, 7),
                                      dy.float().permute(0, 3, 1, 2), stride=2, padding=3)
    assert relerr(dw.view(64, 7, 7, 4)[..., :3], rdw.permute(0, 2, 3, 1)) < 2e-3


def test_batchnorm_fwd_bwd_matches_torch(C):
    N, H, Cc = 4, 8, 64
    x = rnd(N, H, H, Cc, seed=6)
    res = rnd(N, H, H, Cc, seed=7)
    gamma = (torch.rand(Cc) + 0.5).to(dev)
    beta = (torch.randn(Cc) * 0.1).to(dev)
    P = N * H * H
    xf = x.float()
    slab = torch.stack([xf.sum((0, 1, 2)), (xf * xf).sum((0, 1, 2))]).view(1, 2, Cc).contiguous()
    rm, rv = torch.zeros(Cc, device=dev), torch.ones(Cc, device=dev)
    mean, invstd = torch.empty(Cc, device=dev), torch.empty(Cc, device=dev)
    C.bn_finalize(slab, 1, Cc, float(P), 1e-5, 0.1, rm, rv, mean, invstd)
    out = torch.empty_like(x)
    C.bn_apply(x, mean, invstd, gamma, beta, res, True, out)
    # torch reference (fp32, NCHW)
    bn = torch.nn.BatchNorm2d(Cc).to(dev)
    with torch.no_grad():
        bn.weight.copy_(gamma)
        bn.bias.copy_(beta)
    xr = xf.permute(0, 3, 1, 2).clone().requires_grad_(True)
    rr = res.float().permute(0, 3, 1, 2).clone().requires_grad_(True)
    ref = torch.relu(bn(xr) + rr)
    assert relerr(out, ref.permute(0, 2, 3, 1)) < 1e-2
    assert relerr(rm, bn.running_mean) < 1e-5 and relerr(rv, bn.running_var) < 1e-5
    dout = rnd(N, H, H, Cc, seed=8)
    ref.backward(dout.float().permute(0, 3, 1, 2))
    nb = C.bn_bwd_blocks(P, 64)
    s2 = torch.empty(nb, 2 * Cc, device=dev)
    C.bn_bwd_reduce(dout, out, x, mean, invstd, s2, 64)
    sums = torch.empty(2 * Cc, device=dev)
    C.grad_reduce([(s2, 2 * Cc, 0, 2 * Cc, nb, sums, 1.0)])
    dx = torch.empty_like(x)
    dres = torch.empty_like(x)
    C.bn_bwd_apply(dout, out, x, mean, invstd, gamma, sums, float(P), dx, dres)
    assert relerr(dx, xr.grad.permute(0, 2, 3, 1)) < 2e-2
    assert relerr(dres, rr.grad.permute(0, 2, 3, 1)) < 1e-2
    assert relerr(sums[Cc:], bn.weight.grad) < 1e-3 and relerr(sums[:Cc], bn.bias.grad) < 1e-3


def test_pools_and_head(C):
    N, H, Cc = 2, 9, 64
    x = rnd(N, H, H, Cc, seed=9)
    OH = (H - 1) // 2 + 1
    y = torch.empty(N, OH, OH, Cc, dtype=BF, device=dev)
    am = torch.empty(N, OH, OH, Cc, dtype=torch.uint8, device=dev)
    C.maxpool_fwd(x, y, am)
    xr = x.float().permute(0, 3, 1, 2).clone().requires_grad_(True)
    ref = F.max_pool2d(xr, 3, 2, 1)
    assert torch.equal(y.float(), ref.detach().permute(0, 2, 3, 1))
    dy = rnd(N, OH, OH, Cc, seed=10)
    ref.backward(dy.float().permute(0, 3, 1, 2))
    dx = torch.empty_like(x)
    C.maxpool_bwd(dy, am, dx)
    assert relerr(dx, xr.grad.permute(0, 2, 3, 1)) < 1e-2
    a = torch.empty(N, Cc, device=dev)
    C.avgpool_fwd(x, a)
    assert relerr(a, x.float().mean((1, 2))) < 1e-5
    w = torch.randn(1000, Cc, device=dev) * 0.05
    b = torch.randn(1000, device=dev)
    o = torch.empty(N, 1000, device=dev)
    C.sgemm(N, 1000, Cc, a, Cc, 1, w, 1, Cc, o, b, 1.0)
    assert relerr(o, a @ w.t() + b) < 1e-5


def test_resnet18_hip_vs_cpu_fp32():
    """Whole-network gradients of the HIP ResNet-18 vs an fp32 CPU oracle.

    A random-init ResNet-18 amplifies rounding through 20 BatchNorm backwards, so a
    fixed tolerance is meaningless: the bar is the precision floor, i.e. the error
    that torch's own bf16 CPU run of the same network shows against the same fp32
    oracle (scripts/debug_resnet.py prints both columns).  The HIP path must be no
    worse than that floor (plus a small slack) on every parameter."""
    from ddp_amd.models import resnet18
    from ddp_amd.ops import CrossEntropyLoss

    torch.manual_seed(0)
    cpu = resnet18(num_classes=10)
    cpu16 = resnet18(num_classes=10)
    cpu16.load_state_dict(cpu.state_dict())
    gpu = resnet18(num_classes=10).to(dev)
    gpu.load_state_dict(cpu.state_dict())
    x = torch.randn(4, 3, 64, 64)
    y = torch.randint(0, 10, (4,))
    lc = F.cross_entropy(cpu(x), y)
    lc.backward()
    cpu16 = cpu16.to(torch.bfloat16)
    F.cross_entropy(cpu16(x.to(torch.bfloat16)).float(), y).backward()
    lg = CrossEntropyLoss()(gpu(x.to(dev)), y.to(dev))
    lg.backward()
    assert abs(lg.item() - lc.item()) < 5e-2
    bad = []
    for (n, pc), (_, p16), (_, pg) in zip(cpu.named_parameters(), cpu16.named_parameters(),
                                          gpu.named_parameters()):
        e, floor = relerr(pg.grad, pc.grad), relerr(p16.grad.float(), pc.grad)
        if e > 1.25 * floor + 0.03:
            bad.append((n, e, floor))
    assert not bad, bad
    for (n, bc), (_, bg) in zip(cpu.named_buffers(), gpu.named_buffers()):
        if bc.dtype.is_floating_point:
            assert relerr(bg, bc) < 2e-2, n
        else:
            assert torch.equal(bg.cpu(), bc), n
