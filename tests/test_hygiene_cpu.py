"""Small correctness fixes from the round-1 review."""
import pytest
import torch


def test_samples_processed_counts_truncated_epochs():
    from ddp_amd.engine.trainer import samples_processed

    assert samples_processed(1875, 32, 60000) == 60000       # full epoch, ws1
    assert samples_processed(938, 32, 30000) == 30000        # ragged tail (16) included
    assert samples_processed(50, 32, 60000) == 1600          # --max_steps 50
    assert samples_processed(0, 32, 60000) == 0


def test_backend_resolution_never_silently_falls_back(monkeypatch):
    from ddp_amd.parallel import process_group as pg

    monkeypatch.delenv("DDP_AMD_BACKEND", raising=False)
    monkeypatch.delenv("DDP_AMD_DEVICE", raising=False)
    monkeypatch.setattr(torch.cuda, "is_available", lambda: False)
    monkeypatch.setattr(pg, "_gpu_host", lambda: False)
    assert pg.resolve_backend() == "gloo"                    # CPU host: the plumbing config
    assert pg.resolve_backend(device="cpu") == "gloo"
    assert pg.resolve_backend("gloo") == "gloo"
    with pytest.raises(RuntimeError, match="GPU run was requested"):
        pg.resolve_backend(device="gpu")
    with pytest.raises(RuntimeError, match="GPU run was requested"):
        pg.resolve_backend("rccl")
    with pytest.raises(RuntimeError):
        pg.resolve_backend("rccl", device="cpu")
    monkeypatch.setenv("DDP_AMD_DEVICE", "gpu")
    with pytest.raises(RuntimeError):
        pg.resolve_backend()
    monkeypatch.delenv("DDP_AMD_DEVICE")
    # a GPU host whose HIP runtime is unusable: refuse instead of training on the CPU
    monkeypatch.setattr(pg, "_gpu_host", lambda: True)
    with pytest.raises(RuntimeError, match="refusing to fall back"):
        pg.resolve_backend()
    assert pg.resolve_backend(device="cpu") == "gloo"        # explicit CPU run is fine
    # GPU usable: RCCL
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    assert pg.resolve_backend() == "nccl"
    assert pg.resolve_backend("rccl") == "nccl"
    assert pg.resolve_backend(device="gpu") == "nccl"


def test_loaded_momentum_state_means_started():
    """a checkpoint's momentum buffer must resume as a regular update,
    never as the buf = grad initialisation step (the fused engine keys off ``steps``)."""
    from ddp_amd.models import SimpleCNN
    from ddp_amd.ops import FusedSGD

    torch.manual_seed(0)
    m = SimpleCNN()
    opt = FusedSGD(m, lr=0.01, momentum=0.9)
    for p in m.parameters():
        p.grad.normal_()
    opt.step()
    sd = opt.state_dict()
    assert sd["state"]
    m2 = SimpleCNN()
    opt2 = FusedSGD(m2, lr=0.01, momentum=0.9)
    assert opt2.steps == 0
    opt2.load_state_dict(sd)
    assert opt2.steps >= 1 and opt2.momentum_buffer is not None
    assert torch.equal(opt2.momentum_buffer, opt.momentum_buffer)
    # no state -> not started
    opt3 = FusedSGD(SimpleCNN(), lr=0.01, momentum=0.9)
    opt3.load_state_dict(FusedSGD(SimpleCNN(), lr=0.01, momentum=0.9).state_dict())
    assert opt3.steps == 0 and opt3.momentum_buffer is None


@pytest.mark.parametrize("var", ["HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"])
def test_hidden_devices_mean_cpu_run(monkeypatch, var):
    """hiding every GPU through ANY of the visibility variables (empty value) is
    an explicit "no GPU" request - auto mode then trains over gloo instead of raising."""
    from ddp_amd.parallel import process_group as pg

    for v in pg._VISIBILITY_VARS:
        monkeypatch.delenv(v, raising=False)
    monkeypatch.setenv(var, "")
    monkeypatch.setattr(pg.torch.cuda, "is_available", lambda: False)
    assert not pg._gpu_host()
    assert pg.resolve_backend(None, "auto") == "gloo"


def test_module_comm_mapping():
    """--comm reaches the module path: the engine's plan names map onto the
    module reducer's planes."""
    from ddp_amd.engine.trainer import module_comm

    assert module_comm("auto") == "auto" and module_comm("rccl") == "rccl"
    for c in ("xgmi", "xgmi1", "xgmi2", "tune"):
        assert module_comm(c) == "xgmi"
    with pytest.raises(ValueError):
        module_comm("nope")


def test_graph_cache_scoped_to_model():
    """The captured-step cache lives on the model: two models never share
    entries, and it goes away with the model instead of pinning graphs in a global."""
    import gc
    import weakref

    from ddp_amd.engine.trainer import _graph_cache

    a, b = torch.nn.Linear(2, 2), torch.nn.Linear(2, 2)
    ca, cb = _graph_cache(a), _graph_cache(b)
    ca[(4, 2)] = "graph-a"
    assert _graph_cache(a) is ca and cb == {} and ca is not cb
    ref = weakref.ref(ca)
    del a, ca
    gc.collect()
    assert ref() is None


def test_replica_digest_detects_divergence():
    from ddp_amd.engine.trainer import replica_digest
    from ddp_amd.models import SimpleCNN
    from ddp_amd.models.layers import flat_space
    from ddp_amd.ops import FusedSGD

    torch.manual_seed(0)
    m = SimpleCNN()
    fs, opt = flat_space(m), FusedSGD(m, lr=0.01, momentum=0.9)
    d0 = replica_digest(fs, opt)
    assert replica_digest(fs, opt) == d0
    with torch.no_grad():
        fs.params[123] = torch.nextafter(fs.params[123], torch.tensor(1e9))  # one ulp
    assert replica_digest(fs, opt) != d0


def test_no_agent_scope_fences_in_kernels():
    """Round 5: on gfx950 an agent-scope release compiles to `buffer_wbl2 sc1` (a write-back
    of the XCD's whole L2) and an acquire to `buffer_inv sc1` - one per block of an in-launch
    completion count cost the multi-GPU step ~4 us (profiles/r5_dist).  Hand-offs in the
    kernels are relaxed counts after write-through stores + a drain, read with system- or
    agent-scope loads; no kernel source may carry an ordering atomic or a fence."""
    import os
    import re

    root = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc", "kernels")
    pat = re.compile(r"__ATOMIC_(ACQ_REL|RELEASE|ACQUIRE|SEQ_CST)|__threadfence|amdgcn_fence")
    bad = []
    for name in sorted(os.listdir(root)):
        if not name.endswith((".hip", ".h")):
            continue
        with open(os.path.join(root, name)) as f:
            for n, line in enumerate(f, 1):
                code = line.split("//", 1)[0]
                if pat.search(code):
                    bad.append(f"{name}:{n}: {line.strip()}")
    assert not bad, "\n".join(bad)
