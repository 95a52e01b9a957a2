"""The exact-fp32 compute path (``--dtype fp32``): every fp32 kernel
(v_mfma_f32_16x16x4_f32 conv2 forward / data gradient / weight gradient, fp32 conv1 and fc)
against a float64 PyTorch reference of the same op at <= 1e-5 relative error, the
module-path SimpleCNN against the stock fp32 model (the reference's nn.Conv2d / nn.Linear,
/root/reference/model.py:8-16) at <= 1e-4, and the fp32 fused engine's step against the
float64 oracle ``simple_cnn_step_exact``."""
import pytest
import torch

from ddp_amd.ops import reference as R

pytestmark = pytest.mark.gpu
dev = "cuda"
F64 = torch.float64


def rnd(*shape, scale=1.0, seed=0, relu=False):
    g = torch.Generator().manual_seed(seed)
    t = torch.randn(*shape, generator=g) * scale
    if relu:
        t = torch.relu(t)
    return t.to(dev)


def d(t):
    """float64 CPU copy (the oracle runs on the CPU: MIOpen has no fp64 convolutions)."""
    return t.detach().double().cpu()


def relerr(a, b):
    a, b = a.double().cpu(), d(b).cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def test_conv1_fwd_fp32(C):
    B, H, W = 12, 28, 28
    g = torch.Generator().manual_seed(1)
    w = (torch.randn(32, 3, 3, 1, generator=g) * 0.3).to(dev)
    b = (torch.randn(32, generator=g) * 0.1).to(dev)
    x = torch.rand(B, H * W, generator=g).to(dev)
    y = torch.empty(B, H, W, 32, device=dev)
    C.conv1_fwd(x, None, None, 0, 0, w, b, y, B, H, W)
    ref = R.conv1_relu(d(x.view(B, H, W)), d(w), d(b))
    assert relerr(y, ref) < 1e-6


@pytest.mark.parametrize("B,pxt", [(1, 1), (12, 2), (32, 2), (24, 1)])
def test_conv3x3_fwd_fp32(C, B, pxt):
    H = W = 28
    x = rnd(B, H, W, 32, relu=True, seed=2)
    w = rnd(64, 3, 3, 32, scale=0.1, seed=3)
    b = rnd(64, scale=0.1, seed=4)
    y = torch.full((B, H, W, 64), float("nan"), device=dev)
    C.conv3x3_fwd(x, w, b, y, True, None, None, 0, pxt)
    ref = R.conv3x3(d(x), d(w), d(b), relu=True)
    assert relerr(y, ref) < 1e-5
    torch.testing.assert_close(d(y).cpu(), ref.cpu(), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("B", [1, 16, 32])
def test_conv3x3_fwd_fused_fc_fp32(C, B):
    """fp32 fused fc epilogue reads the fc weight in the fp32 FCFRAG order (coalesced)."""
    from ddp_amd.ops.functional import fc_weight_frag, fold_block_partials

    H = W = 28
    x = rnd(B, H, W, 32, relu=True, seed=5)
    w = rnd(64, 3, 3, 32, scale=0.1, seed=6)
    b = rnd(64, scale=0.1, seed=7)
    wfc = rnd(10, H * W, 64, scale=0.01, seed=8)
    bfc = rnd(10, scale=0.1, seed=9)
    y = torch.empty(B, H, W, 64, device=dev)
    nblk = C.conv3x3_dgrad_blocks(B, H, W, 2)
    part = torch.full((nblk, 2, 10), float("nan"), device=dev)
    C.conv3x3_fwd(x, w, b, y, True, fc_weight_frag(wfc, H * W, 64, torch.float32), part, 10, 2)
    logits = fold_block_partials(part, B, H * W, 128) + bfc
    ref = R.fc_nhwc(R.conv3x3(d(x), d(w), d(b)), d(wfc), d(bfc))
    assert relerr(logits, ref) < 1e-5


@pytest.mark.parametrize("mask_dy,mask_x", [(True, False), (False, True), (True, True), (False, False)])
@pytest.mark.parametrize("pxt", [1, 2])
def test_conv3x3_dgrad_fp32(C, mask_dy, mask_x, pxt):
    B, H, W = 12, 28, 28
    dy = rnd(B, H, W, 64, scale=0.5, seed=10)
    yact = rnd(B, H, W, 64, seed=11)
    xact = rnd(B, H, W, 32, seed=12)
    w = rnd(64, 3, 3, 32, scale=0.1, seed=13)
    wt = w.view(64, 9, 32).permute(1, 2, 0).contiguous()
    dx = torch.full((B, H, W, 32), float("nan"), device=dev)
    C.conv3x3_dgrad(dy, yact if mask_dy else None, wt, xact if mask_x else None, dx, pxt)
    g = d(dy) * d(yact > 0) if mask_dy else d(dy)
    ref = R.conv3x3_dgrad(g, d(w))
    if mask_x:
        ref = ref * d(xact > 0)
    assert relerr(dx, ref) < 1e-5


@pytest.mark.parametrize("B,Rrows", [(1, 7), (12, 7), (32, 7), (16, 4), (5, 2)])
def test_conv3x3_wgrad_fp32(C, B, Rrows):
    H = W = 28
    dy = rnd(B, H, W, 64, scale=0.5, seed=14)
    yact = rnd(B, H, W, 64, seed=15)
    x = rnd(B, H, W, 32, relu=True, seed=16)
    nblk = C.conv3x3_wgrad_blocks(B, H, Rrows)
    row = 64 * 9 * 32 + 64
    slab = torch.full((nblk, row), float("nan"), device=dev)
    C.conv3x3_wgrad(dy, yact, x, slab, Rrows)
    gw = torch.empty(64 * 9 * 32, device=dev)
    gb = torch.empty(64, device=dev)
    C.grad_reduce([(slab, row, 0, 64 * 9 * 32, nblk, gw, 1.0), (slab, row, 64 * 9 * 32, 64, nblk, gb, 1.0)])
    g = d(dy) * d(yact > 0)
    rw, rb = R.conv3x3_wgrad(g, d(x))
    assert relerr(gw.view(64, 3, 3, 32), rw) < 1e-5
    assert relerr(gb, rb) < 1e-5
    slab2 = torch.empty_like(slab)
    gw2 = torch.empty_like(gw)
    C.conv3x3_wgrad(dy, yact, x, slab2, Rrows)
    C.grad_reduce([(slab2, row, 0, 64 * 9 * 32, nblk, gw2, 1.0)])
    assert torch.equal(gw, gw2)  # fixed-order split-K: bitwise deterministic


@pytest.mark.parametrize("B", [1, 32])
def test_fc_fwd_bwd_fp32(C, B):
    H = W = 28
    x = rnd(B, H, W, 64, relu=True, seed=17)
    wfc = rnd(10, H * W, 64, scale=0.01, seed=18)
    bfc = rnd(10, scale=0.1, seed=19)
    part = torch.empty(B, 49, 10, device=dev)
    C.fc_partial(x, wfc, part)
    out = torch.empty(B, 10, device=dev)
    C.fc_reduce(part, bfc, out, B, 49, 10)
    assert relerr(out, R.fc_nhwc(d(x), d(wfc), d(bfc))) < 1e-5
    dl = rnd(B, 10, scale=0.1, seed=20)
    for mask in (True, False):
        dx = torch.empty_like(x)
        dw = torch.empty(10, H * W, 64, device=dev)
        C.fc_bwd(dl, x, wfc, dx, dw, 0.5, mask)
        rdx, rdw = R.fc_bwd(d(dl), d(x), d(wfc), mask=mask)
        assert relerr(dx, rdx) < 1e-5
        assert relerr(dw, 0.5 * rdw) < 1e-5


def test_simple_cnn_fp32_module_path_matches_stock_fp32_model():
    """--dtype fp32 module path vs the reference architecture built from stock torch.nn
    layers (fp32, CPU): loss and every gradient within 1e-4."""
    from ddp_amd.models import SimpleCNN, reference_simple_cnn
    from ddp_amd.ops import CrossEntropyLoss

    torch.manual_seed(0)
    ref = reference_simple_cnn()
    gpu = SimpleCNN(compute_dtype=torch.float32).to(dev)
    gpu.load_state_dict(ref.state_dict())
    g0 = torch.Generator().manual_seed(25)
    x = torch.rand(16, 1, 28, 28, generator=g0)
    y = torch.randint(0, 10, (16,), generator=g0)
    loss_r = torch.nn.functional.cross_entropy(ref.forward(x), y)
    loss_r.backward()
    loss_g = CrossEntropyLoss()(gpu(x.to(dev)), y.to(dev))
    loss_g.backward()
    assert abs(loss_g.item() - loss_r.item()) <= 1e-4 * abs(loss_r.item())
    sd_grads = {}
    for n, p in ref.named_parameters():
        sd_grads[n] = p.grad
    # compare in the reference layout (state_dict conversion of our native layouts)
    ours = {}
    for mod_name, mod in (("net.0", gpu.net[0]), ("net.2", gpu.net[2])):
        ours[mod_name + ".weight"] = mod.weight.grad.permute(0, 3, 1, 2)
        ours[mod_name + ".bias"] = mod.bias.grad
    C_, H_, W_ = gpu.fl.in_layout
    ours["fl.weight"] = gpu.fl.weight.grad.permute(0, 2, 1).reshape(10, C_ * H_ * W_)
    ours["fl.bias"] = gpu.fl.bias.grad
    for n, gref in sd_grads.items():
        e = relerr(ours[n], gref)
        assert e < 1e-4, f"{n}: rel err {e:.2e}"


def _engine(B=32, momentum=0.0, fuse_opt=True, use_graph=False, graph_steps=5, dtype="fp32", seed=0,
            fuse_level=1, wgrad_split=1, weight_decay=0.0, l3_fc_role=1, fuse_reduce=None):
    from ddp_amd.data import DeviceMNIST, synthetic_mnist
    from ddp_amd.engine import EngineOptions, FusedSimpleCNNEngine
    from ddp_amd.models import SimpleCNN
    from ddp_amd.ops import FusedSGD

    torch.manual_seed(seed)
    model = SimpleCNN(compute_dtype=torch.float32 if dtype == "fp32" else torch.bfloat16).to(dev)
    opt = FusedSGD(model, lr=0.01, momentum=momentum, weight_decay=weight_decay)
    imgs, labels = synthetic_mnist(2048)
    data = DeviceMNIST(imgs, labels, dev)
    eng = FusedSimpleCNNEngine(model, opt, data, B, 1, 0,
                               opts=EngineOptions(graph_steps=graph_steps, use_graph=use_graph,
                                                  fuse_level=fuse_level, fuse_opt=fuse_opt, dtype=dtype,
                                                  wgrad_split=wgrad_split, l3_fc_role=l3_fc_role,
                                                  fuse_reduce=fuse_reduce))
    eng.refresh()
    return model, opt, eng, imgs, labels


def _native(model):
    return {"w1": model.net[0].weight, "b1": model.net[0].bias, "w2": model.net[2].weight,
            "b2": model.net[2].bias, "wfc": model.fl.weight, "bfc": model.fl.bias}


@pytest.mark.parametrize("B", [32, 12])
@pytest.mark.parametrize("chain", ["level1", "level3"])
def test_fp32_engine_step_matches_float64_oracle(B, chain):
    """One fp32 engine step (separate SGD kernel so the gradient buffer holds the averaged
    gradients): every gradient within 1e-5 of the float64 oracle, loss too - for the
    round-3 level-1 chain and the level-3 chain (dZ2 in the forward, channel-split conv
    backward at two blocks per CU)."""
    kw = dict(fuse_level=1, wgrad_split=1) if chain == "level1" else dict(fuse_level=3, wgrad_split=2)
    model, opt, eng, imgs, labels = _engine(B=B, fuse_opt=False, **kw)
    assert eng.level3 == (chain == "level3")
    assert eng.dtype == "fp32"
    before = {k: v.detach().cpu().clone() for k, v in _native(model).items()}
    eng.fs.grads.fill_(float("nan"))
    eng.run_steps(1)
    eng.synchronize()
    idx = eng.sampler.indices()[:B]
    loss, g = R.simple_cnn_step_exact(before, imgs[idx].double() / 255.0, labels[idx])
    names = {"w1": "net.0.weight", "b1": "net.0.bias", "w2": "net.2.weight", "b2": "net.2.bias",
             "wfc": "fl.weight", "bfc": "fl.bias"}
    for k, name in names.items():
        e = relerr(eng.fs.view(eng.fs.grads, name), g[k])
        assert e < 1e-5, f"{k}: rel err {e:.2e}"
    assert abs(eng.t["loss_hist"][0].item() - loss.item()) < 1e-5 * abs(loss.item())


@pytest.mark.parametrize("momentum", [0.0, 0.9])
def test_fp32_engine_fused_sgd_and_graph_bitwise(momentum):
    """The fp32 engine's fused-SGD epilogues == the separate SGD kernel, graph == eager,
    and the fp32 [tap][ci][co] weight copy stays the exact transpose of the master."""
    m1, o1, e1, _, _ = _engine(momentum=momentum, fuse_opt=False, use_graph=False)
    m2, o2, e2, _, _ = _engine(momentum=momentum, fuse_opt=True, use_graph=True, graph_steps=4)
    e1.run_steps(9)
    e2.run_steps(9)
    e1.synchronize(); e2.synchronize()
    for (n, a), (_, b) in zip(m1.named_parameters(), m2.named_parameters()):
        assert torch.equal(a, b), n
    for e, m in ((e1, m1), (e2, m2)):
        w2 = m.net[2].weight.detach()
        assert torch.equal(e.t["w2t_f32"].view(9, 32, 64), w2.view(64, 9, 32).permute(1, 2, 0))
    assert torch.isfinite(e2.fs.params).all()


def test_fp32_engine_batch_sweep_nan_poisoned():
    for B in (1, 16, 48, 64):
        model, opt, eng, imgs, labels = _engine(B=B, fuse_opt=False)
        for k in ("a2", "dz2", "fc_part", "w2slab", "w1slab"):
            eng.t[k].fill_(float("nan"))
        eng.fs.grads.fill_(float("nan"))
        before = {k: v.detach().cpu().clone() for k, v in _native(model).items()}
        eng.run_steps(1)
        eng.synchronize()
        idx = eng.sampler.indices()[:B]
        _, g = R.simple_cnn_step_exact(before, imgs[idx].double() / 255.0, labels[idx])
        after = {k: v.detach().cpu() for k, v in _native(model).items()}
        for k in g:
            delta = (before[k].double() - after[k].double()) / 0.01
            assert torch.isfinite(delta).all(), (B, k)
            assert relerr(delta, g[k]) < 1e-3, (B, k)  # lr-division of an fp32 update: ~1e-4 noise


@pytest.mark.parametrize("B,momentum,role,fuse_opt,fred", [(32, 0.9, 1, True, 1), (32, 0.0, 1, True, 1),
                                                           (20, 0.9, 1, True, 1), (1, 0.9, 1, True, 1),
                                                           (40, 0.9, 1, True, 1), (32, 0.9, 0, True, 1),
                                                           (32, 0.9, 1, False, 1), (32, 0.9, 1, True, None),
                                                           (32, 0.9, 1, False, None)])
def test_fp32_level3_bitwise_equals_round3_level1(B, momentum, role, fuse_opt, fred):
    """the exact-fp32 step on the level-3 structure - dL and dZ2 in the
    forward, the fc weight gradient + SGD as a role of the conv backward launch (role 1) or
    its own kernel (role 0), both conv backward roles split over input-channel halves at two
    blocks per CU, the fused slab reduction - gives parameters, momentum, losses, the fp32
    weight copies and the step counter bit-identical to round 3's fp32 level-1 chain (one
    conv backward block per row / chunk) after 12 graph-captured steps.  fred None: the fp32
    default, the slab reduction in the separate grad_reduce kernel (faster for fp32, round 6)."""
    kw = dict(B=B, momentum=momentum, weight_decay=1e-4, use_graph=True, graph_steps=4, fuse_opt=fuse_opt)
    m1, o1, e1, _, _ = _engine(fuse_level=1, wgrad_split=1, **kw)
    m3, o3, e3, _, _ = _engine(fuse_level=3, wgrad_split=2, l3_fc_role=role, fuse_reduce=fred, **kw)
    assert e3.level3 and not e1.level3
    e1.run_steps(12)
    e1.synchronize()
    e3.run_steps(12)
    e3.synchronize()
    assert e3.eng.last_level3 and e3.eng.last_fc_role == (role == 1)
    if B == 32:  # two blocks per CU: the 224 wgrad rows fit the reducer budget (fred 1)
        assert e3.eng.last_fused_reduce == (fred == 1)
    for (n, a), (_, b) in zip(m1.named_parameters(), m3.named_parameters()):
        assert torch.equal(a, b), n
    if momentum:
        assert torch.equal(o1.momentum_buffer, o3.momentum_buffer)
    assert torch.equal(e1.t["loss_hist"][:12], e3.t["loss_hist"][:12])
    assert torch.equal(e1.t["step_ctr"], e3.t["step_ctr"])
    assert torch.equal(e1.t["dz2"], e3.t["dz2"])
    for k in ("w2t_f32", "wfc_frag32"):
        assert torch.equal(e1.t[k], e3.t[k]), k
    if not fuse_opt:
        assert torch.equal(e1.fs.grads, e3.fs.grads)
    assert e3.eng.sync_error == 0


def test_fp32_level3_ragged_epoch_bitwise():
    """A whole epoch with a ragged last batch (eager level-3 steps at B < max_batch) on the
    fp32 level-3 chain == the round-3 fp32 level-1 chain, bit for bit."""
    from ddp_amd.data import DeviceMNIST, synthetic_mnist
    from ddp_amd.engine import EngineOptions, FusedSimpleCNNEngine
    from ddp_amd.models import SimpleCNN
    from ddp_amd.ops import FusedSGD

    imgs, labels = synthetic_mnist(1000)
    out = []
    for lvl, split in ((1, 1), (3, 2)):
        torch.manual_seed(0)
        m = SimpleCNN(compute_dtype=torch.float32).to(dev)
        e = FusedSimpleCNNEngine(m, FusedSGD(m, lr=0.01, momentum=0.9), DeviceMNIST(imgs, labels, dev), 32, 1, 0,
                                 opts=EngineOptions(graph_steps=10, fuse_level=lvl, wgrad_split=split, dtype="fp32"))
        e.refresh()
        e.run_epoch(0)
        e.synchronize()
        out.append(e.fs.params.clone())
    assert torch.equal(out[0], out[1])
