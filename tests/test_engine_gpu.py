"""The fused native step engine (csrc/runtime/engine.cpp) on MI355X."""
import pytest
import torch

from ddp_amd.ops import reference as R

pytestmark = pytest.mark.gpu
dev = "cuda"


def _setup(n=2048, B=32, graph_steps=5, use_graph=True, seed=0, lr=0.01, momentum=0.0,
           fuse_level=0, fuse_opt=True, weight_decay=0.0, store_a1=True, **eo):
    from ddp_amd.data import DeviceMNIST, synthetic_mnist
    from ddp_amd.engine import EngineOptions, FusedSimpleCNNEngine
    from ddp_amd.models import SimpleCNN
    from ddp_amd.ops import FusedSGD

    torch.manual_seed(seed)
    model = SimpleCNN().to(dev)
    opt = FusedSGD(model, lr=lr, momentum=momentum, weight_decay=weight_decay)
    imgs, labels = synthetic_mnist(n)
    data = DeviceMNIST(imgs, labels, dev)
    eng = FusedSimpleCNNEngine(model, opt, data, B, 1, 0,
                               opts=EngineOptions(graph_steps=graph_steps, use_graph=use_graph,
                                                  fuse_level=fuse_level, fuse_opt=fuse_opt,
                                                  store_a1=store_a1, **eo))
    eng.refresh()
    return model, opt, data, eng, imgs, labels


def _native(model):
    return {"w1": model.net[0].weight, "b1": model.net[0].bias, "w2": model.net[2].weight,
            "b2": model.net[2].bias, "wfc": model.fl.weight, "bfc": model.fl.bias}


def test_one_step_matches_bf16_reference():
    model, opt, data, eng, imgs, labels = _setup(use_graph=False)
    before = {k: v.detach().cpu().clone() for k, v in _native(model).items()}
    eng.run_steps(1)
    eng.synchronize()
    idx = eng.sampler.indices()[:32]
    x = imgs[idx].float() / 255.0
    loss, g = R.simple_cnn_step_bf16(before, x, labels[idx])
    after = {k: v.detach().cpu() for k, v in _native(model).items()}
    for k in g:
        got = (before[k] - after[k]) / 0.01
        err = (got - g[k]).norm() / g[k].norm()
        assert err < 1e-2, f"{k}: rel err {err:.2e}"
    assert abs(eng.t["loss_hist"][0].item() - loss.item()) < 1e-4


def test_graph_replay_bitwise_equals_eager():
    m1, _, _, e1, _, _ = _setup(use_graph=False)
    m2, _, _, e2, _, _ = _setup(use_graph=True, graph_steps=5)
    e1.run_steps(10)
    e2.run_steps(10)
    e1.synchronize(); e2.synchronize()
    for (n, a), (_, b) in zip(m1.named_parameters(), m2.named_parameters()):
        assert torch.equal(a, b), n


@pytest.mark.parametrize("B", [32, 20])
def test_fuse_level1_bitwise_equals_level0(B):
    """6-kernel step (conv1 recomputed inside conv2 fwd/dgrad/wgrad, xent inside fc_bwd)
    must reproduce the 8-kernel step bit for bit: params, momentum and loss history."""
    m0, _, _, e0, _, _ = _setup(B=B, use_graph=False, momentum=0.9)
    m1, _, _, e1, _, _ = _setup(B=B, use_graph=True, momentum=0.9, fuse_level=1)
    e0.run_steps(7)
    e1.run_steps(7)
    e0.synchronize(); e1.synchronize()
    for (n, a), (_, b) in zip(m0.named_parameters(), m1.named_parameters()):
        assert torch.equal(a, b), n
    assert torch.equal(e0.t["loss_hist"][:7], e1.t["loss_hist"][:7])


@pytest.mark.parametrize("B,opt,momentum,role", [(32, True, 0.9, 1), (32, False, 0.9, 1), (20, True, 0.0, 1),
                                                  (1, True, 0.9, 1), (40, True, 0.9, 1),
                                                  (32, True, 0.9, 0), (20, False, 0.9, 0)])
def test_fuse_level3_bitwise_equals_level1(B, opt, momentum, role):
    """Level 3: the forward computes dZ2 itself (per-image in-launch wait, then dL and
    dZ2 from its fc weight fragments) and the fc weight gradient + SGD runs as a third role
    of the conv backward launch (role) or as its own light kernel (not role).  Parameters,
    momentum, gradients, shadows, losses and the step counter after 10+ graph-captured
    steps must equal the level-1 chain bit for bit, and no in-launch wait
    may time out."""
    kw = dict(B=B, use_graph=True, graph_steps=5, momentum=momentum, weight_decay=1e-4, fuse_opt=opt, store_a1=1)
    m1, o1, _, e1, _, _ = _setup(fuse_level=1, **kw)
    m3, o3, _, e3, _, _ = _setup(fuse_level=3, l3_fc_role=role, **kw)
    assert e3.level3 and not e1.level3
    # one engine at a time: level 3's forward spins on the other blocks of its images, which
    # must all be resident - not shared with another engine's spinning reducers
    e1.run_steps(12)
    e1.synchronize()
    e3.run_steps(12)
    e3.synchronize()
    assert e3.eng.last_level3 and e3.eng.last_fc_role == (role > 0)
    for (n, a), (_, b) in zip(m1.named_parameters(), m3.named_parameters()):
        assert torch.equal(a, b), n
    if momentum:
        assert torch.equal(o1.momentum_buffer, o3.momentum_buffer)
    assert torch.equal(e1.t["loss_hist"][:12], e3.t["loss_hist"][:12])
    assert torch.equal(e1.t["step_ctr"], e3.t["step_ctr"])
    assert torch.equal(e1.t["dz2"], e3.t["dz2"])
    for k in ("w2_bf16", "w2t_bf16", "wfc_frag"):  # (level 3 never reads / refreshes wfc_bf16)
        assert torch.equal(e1.t[k], e3.t[k]), k
    if not opt:  # the flat SGD kernel reads the reduced gradients
        assert torch.equal(e1.fs.grads, e3.fs.grads)
    assert e3.eng.sync_error == 0


@pytest.mark.parametrize("B,n", [(32, 1000), (64, 2000)])
def test_fuse_level3_ragged_epoch(B, n):
    """A whole epoch with a ragged last batch (eager level-3 step at B = 8 / 16, counters of
    fewer images), bit-identical to level 1 - also at the README's B = 64,
    whose 392 forward blocks exceed the resident capacity: a block waits only for its own
    image's blocks, which in-order dispatch always provides (conv3x3_fwd_dz_fits), and the
    fc role holds 64 rows - 2 kernels per step."""
    m1, _, _, e1, _, _ = _setup(n=n, B=B, graph_steps=10, fuse_level=1, momentum=0.9)
    m3, _, _, e3, _, _ = _setup(n=n, B=B, graph_steps=10, fuse_level=3, momentum=0.9)
    losses = ([], [])
    for e, ls in ((e1, losses[0]), (e3, losses[1])):  # one engine at a time (see above)
        e.run_epoch(0, on_loss=lambda b, l, ls=ls: ls.append(l), log_every=5)
        e.run_epoch(1)
        e.synchronize()
    assert e3.level3 and e3.eng.level3_active(n % B) and e3.eng.last_level3 and e3.eng.last_fc_role
    for (k, a), (_, b) in zip(m1.named_parameters(), m3.named_parameters()):
        assert torch.equal(a, b), k
    assert losses[0] == losses[1]
    assert e3.eng.sync_error == 0


@pytest.mark.parametrize("dtype,B,opt", [("bf16", 32, True), ("bf16", 20, True), ("bf16", 64, False),
                                         ("fp32", 32, True), ("fp32", 20, False)])
def test_fused_reduce_bitwise_equals_grad_reduce(dtype, B, opt):
    """The conv backward launch that also reduces the split-K slabs (wgrad blocks, after an
    in-launch arrival count, sc1 loads, grad_reduce's fixed order) must equal the separate
    grad_reduce kernel bit for bit - with the fused optimizer (opt) and without it (flat
    SGD kernel after the reduction)."""
    kw = dict(B=B, use_graph=True, momentum=0.9, weight_decay=1e-4, fuse_level=1, fuse_opt=opt,
              store_a1=0, dtype=dtype)
    m1, o1, _, e1, _, _ = _setup(fuse_reduce=False, **kw)
    m2, o2, _, e2, _, _ = _setup(fuse_reduce=2, **kw)
    e1.run_steps(11)
    e2.run_steps(11)
    e1.synchronize(); e2.synchronize()
    for (n, a), (_, b) in zip(m1.named_parameters(), m2.named_parameters()):
        assert torch.equal(a, b), n
    assert torch.equal(o1.momentum_buffer, o2.momentum_buffer)
    assert torch.equal(e1.fs.grads, e2.fs.grads)
    assert torch.equal(e1.t["loss_hist"][:11], e2.t["loss_hist"][:11])
    assert torch.equal(e1.t["step_ctr"], e2.t["step_ctr"])
    assert e2.eng.sync_error == 0
    assert not e1.eng.last_fused_reduce
    # the wgrad blocks (the reducers) fuse while they fit the resident capacity (single
    # process: all of it): bf16 (2 blocks per CU) and fp32 (1 block per CU, 4-row chunks:
    # 224 slab rows at B = 32) - bitwise equal to the separate kernel either way
    assert e2.eng.last_fused_reduce
    print(f"fused reduce {dtype} B={B}: {e2.eng.last_fused_reduce}")


@pytest.mark.parametrize("B,fred,store_a1", [(32, True, 0), (32, False, 0), (20, True, 0), (64, True, 0), (32, True, 1),
                                             (32, True, 2)])
def test_wgrad_channel_split_bitwise(B, fred, store_a1):
    """Two wgrad blocks per slab row (input-channel halves, XCD-paired block order; B=20
    gives a row count that is not a multiple of 8 - the adjacent-pair order) must write
    the same slab rows as one block per row: parameters, momentum, gradients and losses
    bit-identical after 11 steps, with the fused in-launch reduction and without it,
    recomputing a1 (store_a1 0) or loading it (2)."""
    kw = dict(B=B, use_graph=True, momentum=0.9, weight_decay=1e-4, fuse_level=1, store_a1=store_a1,
              fuse_reduce=fred)
    m1, o1, _, e1, _, _ = _setup(wgrad_split=1, **kw)
    m2, o2, _, e2, _, _ = _setup(wgrad_split=2, **kw)
    e1.run_steps(11)
    e2.run_steps(11)
    e1.synchronize(); e2.synchronize()
    for (n, a), (_, b) in zip(m1.named_parameters(), m2.named_parameters()):
        assert torch.equal(a, b), n
    assert torch.equal(o1.momentum_buffer, o2.momentum_buffer)
    assert torch.equal(e1.fs.grads, e2.fs.grads)
    assert torch.equal(e1.t["loss_hist"][:11], e2.t["loss_hist"][:11])
    assert e2.eng.sync_error == 0
    assert e1.eng.last_fused_reduce == e2.eng.last_fused_reduce


@pytest.mark.parametrize("momentum,wd", [(0.0, 0.0), (0.9, 1e-4)])
def test_fused_optimizer_bitwise_equals_sgd_kernel(momentum, wd):
    """Single-process steps apply SGD in the fc_bwd / grad_reduce epilogues; the result
    must equal the separate flat SGD kernel bit for bit (same sgd_one, same values)."""
    m1, o1, _, e1, _, _ = _setup(use_graph=True, momentum=momentum, weight_decay=wd, fuse_level=1,
                                 fuse_opt=False)
    m2, o2, _, e2, _, _ = _setup(use_graph=True, momentum=momentum, weight_decay=wd, fuse_level=1,
                                 fuse_opt=True)
    e1.run_steps(11)
    e2.run_steps(11)
    e1.synchronize(); e2.synchronize()
    for (n, a), (_, b) in zip(m1.named_parameters(), m2.named_parameters()):
        assert torch.equal(a, b), n
    if momentum:
        assert torch.equal(o1.momentum_buffer, o2.momentum_buffer)
    for k in ("w2_bf16", "w2t_bf16", "wfc_bf16", "wfc_frag"):
        assert torch.equal(e1.t[k], e2.t[k]), k
    assert torch.equal(e1.t["step_ctr"], e2.t["step_ctr"])


@pytest.mark.parametrize("store_a1", [1, 2])
def test_stored_a1_bitwise_equals_recomputed_a1(store_a1):
    """Level 1 either stores a1 in the forward for the conv backward or recomputes conv1
    there from the compact batch; both must give the same parameters bit for bit."""
    m1, _, _, e1, _, _ = _setup(use_graph=True, fuse_level=1, store_a1=store_a1, momentum=0.9)
    m2, _, _, e2, _, _ = _setup(use_graph=True, fuse_level=1, store_a1=0, momentum=0.9)
    e1.run_steps(11)
    e2.run_steps(11)
    e1.synchronize(); e2.synchronize()
    for (n, a), (_, b) in zip(m1.named_parameters(), m2.named_parameters()):
        assert torch.equal(a, b), n


def test_fuse_level1_one_step_matches_bf16_reference():
    model, opt, data, eng, imgs, labels = _setup(use_graph=False, fuse_level=1)
    before = {k: v.detach().cpu().clone() for k, v in _native(model).items()}
    eng.run_steps(1)
    eng.synchronize()
    idx = eng.sampler.indices()[:32]
    loss, g = R.simple_cnn_step_bf16(before, imgs[idx].float() / 255.0, labels[idx])
    after = {k: v.detach().cpu() for k, v in _native(model).items()}
    for k in g:
        got = (before[k] - after[k]) / 0.01
        err = (got - g[k]).norm() / g[k].norm()
        assert err < 1e-2, f"{k}: rel err {err:.2e}"
    assert abs(eng.t["loss_hist"][0].item() - loss.item()) < 1e-4


@pytest.mark.parametrize("fuse_level", [0, 1, 3])
@pytest.mark.parametrize("B", [1, 12, 16, 24, 48, 64])
def test_engine_batch_sweep_nan_poisoned(B, fuse_level):
    """SURVEY §4.1 batch sizes; every intermediate buffer starts as NaN so a kernel that
    reads something its producer did not write shows up as a non-finite gradient."""
    model, opt, data, eng, imgs, labels = _setup(B=B, use_graph=False, fuse_level=fuse_level)
    for k in ("a1", "a2", "dz2", "dz1", "fc_part", "dlogits", "loss_rows", "w2slab", "w1slab"):
        eng.t[k].fill_(float("nan"))
    eng.fs.grads.fill_(float("nan"))
    before = {k: v.detach().cpu().clone() for k, v in _native(model).items()}
    eng.run_steps(1)
    eng.synchronize()
    idx = eng.sampler.indices()[:B]
    loss, g = R.simple_cnn_step_bf16(before, imgs[idx].float() / 255.0, labels[idx])
    after = {k: v.detach().cpu() for k, v in _native(model).items()}
    for k in g:
        got = (before[k] - after[k]) / 0.01
        assert torch.isfinite(got).all(), k
        err = (got - g[k]).norm() / g[k].norm()
        assert err < 1e-2, f"B={B} {k}: rel err {err:.2e}"
    assert abs(eng.t["loss_hist"][0].item() - loss.item()) < 1e-4


def test_run_epoch_ragged_and_logging():
    model, opt, data, eng, _, _ = _setup(n=1000, B=32, graph_steps=10)
    seen = []
    n = eng.run_epoch(0, on_loss=lambda b, l: seen.append((b, l)), log_every=10)
    eng.synchronize()
    assert n == 32  # ceil(1000/32): 31 full + ragged 8
    assert [b for b, _ in seen] == [0, 10, 20, 30]
    assert all(torch.isfinite(torch.tensor(l)) for _, l in seen)
    assert torch.isfinite(eng.fs.params).all()
    # the loss goes down on the learnable synthetic set
    for e in range(1, 4):
        eng.run_epoch(e)
    eng.synchronize()
    assert eng.t["loss_hist"][0].item() < seen[0][1]


def test_momentum_engine_matches_module_sgd_semantics():
    model, opt, data, eng, _, _ = _setup(use_graph=True, graph_steps=4, momentum=0.9)
    seen = []
    eng.run_epoch(0, on_loss=lambda b, l: seen.append(l), log_every=16)
    eng.synchronize()
    assert opt.momentum_buffer is not None and torch.isfinite(opt.momentum_buffer).all()
    sd = opt.state_dict()
    assert set(sd["state"].keys()) == set(range(6))


def test_module_ddp_world1_rccl(tmp_path):
    """Our DDP (native C++ reducer + RCCL comm) at ws=1 leaves grads unchanged."""
    import torch.distributed as dist

    from ddp_amd.models import SimpleCNN
    from ddp_amd.ops import CrossEntropyLoss
    from ddp_amd.parallel import DistributedDataParallel, free_port

    dist.init_process_group("nccl", rank=0, world_size=1,
                            store=dist.HashStore(),
                            device_id=torch.device("cuda", 0))
    try:
        torch.manual_seed(0)
        a = SimpleCNN().to(dev)
        b = SimpleCNN().to(dev)
        b.load_state_dict(a.state_dict())
        ddp = DistributedDataParallel(b)
        x = torch.rand(8, 1, 28, 28, device=dev)
        y = torch.randint(0, 10, (8,), device=dev)
        CrossEntropyLoss()(a(x), y).backward()
        CrossEntropyLoss()(ddp(x), y).backward()
        torch.cuda.synchronize()
        for (n, p), (_, q) in zip(a.named_parameters(), b.named_parameters()):
            torch.testing.assert_close(q.grad, p.grad, rtol=0, atol=0)
        assert ddp.allreduce_buckets_launched == 2
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("fuse_level", [1, 3])
def test_engine_rccl_allreduce_inside_graph_world1(fuse_level):
    """Bucket all-reduces over RCCL on the comm stream, captured in the hipGraph with their
    events (RCCL at world size 1 is the identity): bitwise equal to the comm-free run.
    comm="rccl" forces the RCCL data plane (the default "auto" would pick the xGMI kernels
    even at world size 1) - the plane the 8-GPU run falls back to."""
    import torch.distributed as dist

    from ddp_amd.data import DeviceMNIST, synthetic_mnist
    from ddp_amd.engine import EngineOptions, FusedSimpleCNNEngine
    from ddp_amd.models import SimpleCNN
    from ddp_amd.ops import FusedSGD
    from ddp_amd.parallel import free_port, native_comm

    dist.init_process_group("nccl", rank=0, world_size=1,
                            store=dist.HashStore(),
                            device_id=torch.device("cuda", 0))
    try:
        comm = native_comm()
        imgs, labels = synthetic_mnist(2048)
        data = DeviceMNIST(imgs, labels, dev)
        out = []
        for force in (False, True):
            torch.manual_seed(0)
            m = SimpleCNN().to(dev)
            e = FusedSimpleCNNEngine(m, FusedSGD(m, lr=0.01), data, 32, 1, 0, comm,
                                     EngineOptions(graph_steps=5, force_allreduce=force, comm="rccl",
                                                   fuse_level=fuse_level))
            assert e.comm_kind == ("rccl" if force else "none")
            assert e.level3 == (fuse_level == 3)
            e.refresh()
            e.run_steps(10)
            e.synchronize()
            assert e.eng.sync_error == 0
            out.append(e.fs.params.clone())
        assert torch.equal(out[0], out[1])
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("fuse_level", [1, 3])
@pytest.mark.parametrize("use_graph", [False, True])
def test_engine_xgmi_world1_beside_fused_reduce(fuse_level, use_graph):
    """The direct xGMI all-reduce kernels at world size 1 (forced) on the comm stream, next
    to the conv backward's fused in-launch slab reduction (its reducers spin beside the
    all-reduce kernel of the fc bucket): eager and graph-captured runs equal the comm-free
    run bit for bit, and the reduction really was fused."""
    import torch.distributed as dist

    from ddp_amd.data import DeviceMNIST, synthetic_mnist
    from ddp_amd.engine import EngineOptions, FusedSimpleCNNEngine
    from ddp_amd.models import SimpleCNN
    from ddp_amd.ops import FusedSGD
    from ddp_amd.parallel import free_port

    dist.init_process_group("gloo", rank=0, world_size=1, store=dist.HashStore())
    try:
        imgs, labels = synthetic_mnist(2048)
        data = DeviceMNIST(imgs, labels, dev)
        out = []
        for force in (False, True):
            torch.manual_seed(0)
            m = SimpleCNN().to(dev)
            e = FusedSimpleCNNEngine(m, FusedSGD(m, lr=0.01, momentum=0.9), data, 32, 1, 0, None,
                                     EngineOptions(graph_steps=5, use_graph=use_graph, force_allreduce=force,
                                                   comm="xgmi", fuse_level=fuse_level))
            if force:
                assert e.comm_kind.startswith("xgmi"), e.comm_kind
            e.refresh()
            e.run_steps(10)
            e.synchronize()
            assert e.eng.last_fused_reduce
            assert e.eng.sync_error == 0
            out.append(e.fs.params.clone())
        assert torch.equal(out[0], out[1])
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("corrupt,stall", [(False, False), (True, False), (False, True)])
def test_verify_chain_world1_forced(corrupt, stall):
    """VERDICT r3 #3a on one GPU: the start-up chain check (production = level 3 + fused
    slab reduction + the xGMI kernels forced at world size 1; conservative = level 1 +
    grad_reduce over the same plane) passes bitwise and restores its snapshot exactly (the
    following training equals a run without the check); with a forced one-ulp disagreement
    the engine downgrades to the conservative chain and trains to the same bits."""
    import torch.distributed as dist

    from ddp_amd.data import DeviceMNIST, synthetic_mnist
    from ddp_amd.engine import EngineOptions, FusedSimpleCNNEngine
    from ddp_amd.models import SimpleCNN
    from ddp_amd.ops import FusedSGD
    from ddp_amd.parallel import free_port

    dist.init_process_group("gloo", rank=0, world_size=1, store=dist.HashStore())
    try:
        imgs, labels = synthetic_mnist(2048)
        data = DeviceMNIST(imgs, labels, dev)
        out = []
        for check in (False, True):
            torch.manual_seed(0)
            m = SimpleCNN().to(dev)
            e = FusedSimpleCNNEngine(m, FusedSGD(m, lr=0.01, momentum=0.9), data, 32, 1, 0, None,
                                     EngineOptions(graph_steps=5, force_allreduce=True, comm="xgmi"))
            assert e.level3 and e.comm_kind.startswith("xgmi")
            e.refresh()
            if check and stall:
                # a long kernel queued on the production stream in front of every
                # snapshot restore - the conservative engine (its own stream) must still start
                # from the restored state, not race the copies
                orig = e.start_epoch

                def slow_start(ep, _orig=orig, _e=e):
                    with torch.cuda.stream(_e.stream):
                        torch.cuda._sleep(40_000_000)
                    _orig(ep)

                e.start_epoch = slow_start
            if check:
                kept = e.verify_chain(_corrupt_rank=0 if corrupt else None)
                assert e.chain_check["ran"]
                assert kept == (not corrupt), e.chain_check
                assert e.chain_check["identical_here"] == (not corrupt)
                assert e.level3 == (not corrupt) and (e.cfg["fuse_level"] == (3 if not corrupt else 1))
                # the independent host oracle ran on the production chain's step 1 and agreed
                assert e.chain_check["oracle"]["ran"] and e.chain_check["oracle"]["mismatches"] == 0, e.chain_check
                assert e.chain_check["pair"], e.chain_check  # the dist_mode 3 pair launch was checked
            e.run_steps(12)
            e.synchronize()
            assert e.eng.sync_error == 0
            out.append((e.fs.params.clone(), e.opt.momentum_buffer.clone()))
        assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("comm", ["xgmi", "xgmi2"])
def test_verify_chain_covers_the_step_head(comm):
    """dist_mode 4's step head exists only in captured graphs: the start-up check runs the
    production chain's steps as a graph (momentum-init step eager), so at least one step head
    is compared with the conservative chain before training commits to it.  "xgmi": the conv
    bucket one-shot (conv2's tap-transposed shadow written after its count); "xgmi2": both
    buckets two-shot (every shadow in the SGD pass)."""
    import torch.distributed as dist

    from ddp_amd.data import DeviceMNIST, synthetic_mnist
    from ddp_amd.engine import EngineOptions, FusedSimpleCNNEngine
    from ddp_amd.models import SimpleCNN
    from ddp_amd.ops import FusedSGD

    dist.init_process_group("gloo", rank=0, world_size=1, store=dist.HashStore())
    try:
        imgs, labels = synthetic_mnist(2048)
        torch.manual_seed(0)
        m = SimpleCNN().to(dev)
        e = FusedSimpleCNNEngine(m, FusedSGD(m, lr=0.01, momentum=0.9), DeviceMNIST(imgs, labels, dev), 32, 1, 0,
                                 None, EngineOptions(graph_steps=5, force_allreduce=True, comm=comm, dist_mode=4))
        e.refresh()
        assert e.eng.overlap_active()
        assert e.verify_chain(), e.chain_check
        assert e.chain_check["step_heads_checked"] >= 1 and e.chain_check["oracle"]["mismatches"] == 0, e.chain_check
        e.run_steps(10)
        e.synchronize()
        assert e.eng.graph_heads == 4 and e.eng.sync_error == 0
    finally:
        dist.destroy_process_group()


def test_verify_chain_oracle_downgrades_to_rccl():
    """a one-ulp error in the xGMI-reduced gradient (injected into the bucket
    the production chain reduced) is caught by the host oracle - not by the conservative
    chain, which shares the xGMI code - and the engine moves to RCCL, then trains to the
    comm-free chain's bits (world size 1: RCCL's one-rank sum is exact)."""
    import torch.distributed as dist

    from ddp_amd.data import DeviceMNIST, synthetic_mnist
    from ddp_amd.engine import EngineOptions, FusedSimpleCNNEngine
    from ddp_amd.models import SimpleCNN
    from ddp_amd.ops import FusedSGD
    from ddp_amd.parallel import native_comm

    dist.init_process_group("nccl", rank=0, world_size=1, store=dist.HashStore(),
                            device_id=torch.device("cuda", 0))
    try:
        imgs, labels = synthetic_mnist(2048)
        data = DeviceMNIST(imgs, labels, dev)
        out = []
        for force in (False, True):
            torch.manual_seed(0)
            m = SimpleCNN().to(dev)
            e = FusedSimpleCNNEngine(m, FusedSGD(m, lr=0.01, momentum=0.9), data, 32, 1, 0, native_comm(),
                                     EngineOptions(graph_steps=5, force_allreduce=force, comm="xgmi"))
            e.refresh()
            if force:
                assert e.comm_kind.startswith("xgmi")
                kept = e.verify_chain(_corrupt_oracle_rank=0)
                cc = e.chain_check
                assert not kept and cc["identical_all"] and not cc["oracle_ok_all"], cc
                assert cc["oracle"]["mismatches"] == 1, cc
                assert e.comm_kind == "rccl" and e.xgmi is None
            e.run_steps(12)
            e.synchronize()
            out.append((e.fs.params.clone(), e.opt.momentum_buffer.clone()))
        assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])
    finally:
        dist.destroy_process_group()


def test_comm_tune_rccl_candidates_world1():
    """``--comm tune`` also times RCCL algorithm / protocol variants - one
    fresh communicator per (NCCL_ALGO, NCCL_PROTO) candidate, timed only if it initialised -
    and the engine trains on whichever plane won (bitwise the comm-free run at world 1)."""
    import torch.distributed as dist

    from ddp_amd.data import DeviceMNIST, synthetic_mnist
    from ddp_amd.engine import EngineOptions, FusedSimpleCNNEngine
    from ddp_amd.models import SimpleCNN
    from ddp_amd.ops import FusedSGD
    from ddp_amd.parallel import free_port, native_comm
    from ddp_amd.parallel.xgmi import rccl_candidate_comms

    dist.init_process_group("nccl", rank=0, world_size=1, store=dist.HashStore(),
                            device_id=torch.device("cuda", 0))
    try:
        variants = rccl_candidate_comms(0, 1)
        assert len(variants) >= 1, variants
        t = torch.ones(1000, device=dev)
        for name, c in variants.items():
            assert name.startswith("rccl:")
            c.all_reduce(t)
        torch.cuda.synchronize()
        assert torch.equal(t, torch.ones(1000, device=dev))
        imgs, labels = synthetic_mnist(2048)
        data = DeviceMNIST(imgs, labels, dev)
        out = []
        for force in (False, True):
            torch.manual_seed(0)
            m = SimpleCNN().to(dev)
            e = FusedSimpleCNNEngine(m, FusedSGD(m, lr=0.01), data, 32, 1, 0, native_comm(),
                                     EngineOptions(graph_steps=5, force_allreduce=force, comm="tune"))
            if force:
                assert e.allreduce_us and any(k.startswith("rccl:") for k in e.allreduce_us), e.allreduce_us
                assert e.comm_kind in ("xgmi", "xgmi1") or e.comm_kind.startswith("rccl"), e.comm_kind
            e.refresh()
            e.run_steps(10)
            e.synchronize()
            out.append(e.fs.params.clone())
        assert torch.equal(out[0], out[1])
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("plane,dtype", [("xgmi", "bf16"), ("xgmi", "fp32"), ("rccl", "bf16")])
def test_dist_chains_bitwise_world1(plane, dtype, monkeypatch):
    """every multi-GPU step chain trains to the same bits as the comm-free
    one-GPU chain, at world size 1 with the all-reduces forced and the 8-rank bucket plan (fc
    bucket two-shot, conv bucket one-shot), graph-replayed, with momentum (the fused SGD of
    the xGMI all-gather updates the momentum buffer too) and a ragged last batch:
    dist_mode 3 (default) - both buckets' all-reduces in one launch behind the conv backward
    (xGMI; 3 kernels per step, xgmi_allreduce_pair), 2 - the in-launch all-reduce (xGMI; 2
    kernels per step, engine.cpp make_xar; its grid does not fit the GPU at once, so it needs
    the in-order-dispatch opt-in DDP_AMD_L3_INORDER=1 - without it the bucket kernels run,
    "inlaunch_fb"), 1 - fc_bwd + the fc bucket forked beside the conv backward, 0 - the
    round-4 serial order, 4 - the step head (bf16: the pair launch of step k also runs step
    k + 1's forward, conv3x3.hip step_head_kernel; fp32: mode 3's chain)."""
    import torch.distributed as dist

    from ddp_amd.data import DeviceMNIST, synthetic_mnist
    from ddp_amd.engine import EngineOptions, FusedSimpleCNNEngine
    from ddp_amd.models import SimpleCNN
    from ddp_amd.ops import FusedSGD
    from ddp_amd.parallel import free_port, native_comm

    # (an in-process store: no TCP port to race for)
    if plane == "rccl":
        dist.init_process_group("nccl", rank=0, world_size=1, store=dist.HashStore(),
                                device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo", rank=0, world_size=1, store=dist.HashStore())
    try:
        comm = native_comm() if plane == "rccl" else None
        imgs, labels = synthetic_mnist(1000)  # 31 full batches + a ragged one of 8
        data = DeviceMNIST(imgs, labels, dev)
        out = {}
        # (dist_mode 4 runs the 256-thread forward, pxt_fwd 1, whose per-block partial logits
        # group the fc sum differently: it is compared with the comm-free chain at pxt 1)
        modes = (("local", False, 3), ("serial", True, 0), ("fork", True, 1), ("inlaunch", True, 2),
                 ("inlaunch_fb", True, 2), ("pair", True, 3)) + \
            ((("local_pf1", False, 3),) if dtype == "bf16" else ()) + (("head", True, 4),)
        for tag, force, mode in modes:
            if tag == "inlaunch":
                monkeypatch.setenv("DDP_AMD_L3_INORDER", "1")
            else:
                monkeypatch.delenv("DDP_AMD_L3_INORDER", raising=False)
            torch.manual_seed(0)
            m = SimpleCNN(compute_dtype=torch.float32 if dtype == "fp32" else torch.bfloat16).to(dev)
            e = FusedSimpleCNNEngine(m, FusedSGD(m, lr=0.01, momentum=0.9), data, 32, 1, 0, comm,
                                     EngineOptions(graph_steps=5, force_allreduce=force, comm=plane,
                                                   dist_mode=mode, plan_world=8 if force else None,
                                                   dtype=dtype, pxt_fwd=1 if tag == "local_pf1" else 2))
            if force:
                assert e.comm_kind.startswith(plane), e.comm_kind
                assert len(e.ranges) == 2  # the 8-rank plan: [fc], [conv]
            assert e.level3
            e.refresh()
            e.run_epoch(0)  # (its ragged last step of 8 reduces its slabs apart: bucket kernels)
            e.run_steps(3)  # full batches again: the in-launch all-reduce runs
            e.synchronize()
            assert e.eng.sync_error == 0 and e.eng.last_level3
            if tag != "inlaunch_fb":  # (in-launch iff its whole grid fits this GPU at once)
                assert e.eng.last_xar == (tag == "inlaunch" and plane == "xgmi"), tag
            assert e.eng.last_pair == (tag in ("pair", "head") and plane == "xgmi"), tag
            # dist_mode 4 (bf16): the captured graph's pair launches carried the next forward
            head = tag == "head" and plane == "xgmi" and dtype == "bf16"
            assert e.eng.overlap_active() == head, tag
            e.run_steps(5)  # one whole graph replay (dist_mode 4: its pair launches carry forwards)
            e.synchronize()
            # a 5-step graph: 4 step heads ([fwd 0] [bwd 0] [pair 0 + fwd 1] ... [bwd 4] [pair 4])
            assert e.eng.graph_heads == (4 if head else 0) and e.eng.sync_error == 0, (tag, e.eng.graph_heads)
            out[tag] = (e.fs.params.clone(), e.opt.momentum_buffer.clone())
        for tag, _, mode in modes[1:]:
            if tag == "local_pf1":
                continue
            ref = "local_pf1" if (mode == 4 and dtype == "bf16") else "local"
            assert torch.equal(out[tag][0], out[ref][0]), tag
            assert torch.equal(out[tag][1], out[ref][1]), tag
    finally:
        dist.destroy_process_group()


def test_rccl_premul_sum_world1_eager_and_graph():
    """the module-path reducer's RCCL plane folds DDP's 1/ws prescale into the
    reduction (RCCL pre-multiplied SUM, Comm::all_reduce_premul) instead of a separate
    scale pass; at world size 1 the result is exactly x * scale (fp32 multiply), eagerly and
    replayed from a captured graph (the host-immediate scalar is captured by value).
    (RCCL 2.26's one-rank path leaves the last n % 4 elements of a large buffer unscaled -
    scripts/premul_probe.py, profiles/r5_dist; since round 6 the reducer takes the
    pre-multiplied SUM only when opted in, DDP_AMD_RCCL_PREMUL=1, and only for 16-byte-aligned
    buckets of whole quads - no multi-rank run has pinned it against scale + SUM)"""
    import torch.distributed as dist

    from ddp_amd.parallel import free_port, native_comm

    # (an in-process store: no TCP port to race for)
    dist.init_process_group("nccl", rank=0, world_size=1, store=dist.HashStore(), device_id=torch.device("cuda", 0))
    try:
        comm = native_comm()
        x = torch.randn(100_000, device=dev)
        s = 1.0 / 3.0
        want = x * torch.tensor(s, dtype=torch.float32, device=dev)
        y = x.clone()
        comm.all_reduce_premul(y, s)
        torch.cuda.synchronize()
        assert torch.equal(y, want)
        z = x.clone()
        g = torch.cuda.CUDAGraph()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            with torch.cuda.graph(g):
                comm.all_reduce_premul(z, s)
        torch.cuda.current_stream().wait_stream(side)
        z.copy_(x)
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(z, want)
    finally:
        dist.destroy_process_group()
