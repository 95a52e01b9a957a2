"""Per-rank training entry point - the reference's ``ddp_train`` (train_ddp.py:17-212).

Same phases, same log lines, same checkpoint/resume contract,
with the reference's bugs fixed and the hot loop replaced:

* GPU (default): the native fused step engine - 2 HIP kernels per step on one GPU
  (fuse level 3), plus the light fc weight-gradient kernel and one direct-xGMI (or RCCL)
  all-reduce per gradient bucket on several, hipGraph-replayed, dataset resident in HBM;
* GPU ``--engine module``: the module path (HIP autograd Functions + our DDP with
  the native C++ reducer) - the reference's loop shape, kernel-for-kernel on HIP;
* GPU with ``--backend gloo --device gpu``: the same GPU paths with a gloo control plane
  and the direct xGMI data plane - several ranks may share one GPU, which rehearses the
  multi-GPU trainer (checkpoint / resume, bucket all-reduces) on a single device;
* CPU: gloo + the reference's loop over a DataLoader (BASELINE config 1).

``model="resnet18"`` (BASELINE config 5) trains torchvision-layout ResNet-18 on
synthetic ImageNet-shaped data through the module path (GPU: the HIP ResNet Functions,
our DDP and the native reducer, optionally the whole step in one hipGraph; CPU: the
PyTorch oracle), with the same launcher, logging, checkpoint and resume contract.
"""
from __future__ import annotations

import dataclasses
import os
import time

import torch
import torch.distributed as dist

from ..data import (DeviceImageLoader, DeviceImages, DeviceMNIST, DeviceMNISTLoader, get_dataloader,
                    load_mnist, synthetic_imagenet)
from ..models import SimpleCNN, resnet18
from ..models.layers import buffer_space, flat_space
from ..ops import CrossEntropyLoss, FusedSGD
from ..parallel import DistributedDataParallel as DDP
from ..parallel import cleanup, local_rank, native_comm, setup
from ..utils.checkpoint import resume, save_checkpoint


@dataclasses.dataclass
class TrainOptions:
    lr: float = 0.01
    momentum: float = 0.0
    weight_decay: float = 0.0
    backend: str | None = None        # rccl|nccl|gloo (default: rccl on GPU, gloo on CPU)
    device: str | None = None         # auto|gpu|cpu: "gpu" fails loudly without a usable HIP device
    engine: str = "fused"             # fused | module   (GPU only)
    data: str = "auto"                # auto | mnist | synthetic
    data_root: str = "./data"
    checkpoint_dir: str = "./checkpoints"
    save: bool = True
    seed: int | None = 0
    log_every: int = 100
    graph_steps: int = 100
    bucket_cap_mb: float = 25.0
    num_workers: int = 2
    max_steps: int | None = None      # stop each epoch early (smoke tests)
    metrics_json: str | None = None   # append per-epoch throughput records here
    fault: tuple | None = None        # (epoch, step, rank|-1): simulate a crash there (resume tests)
    fuse_level: int | None = None     # fused engine fusion level (None: engine default)
    comm: str = "auto"                # fused engine bucket all-reduce: auto/xgmi (direct kernel) | rccl
    # fused engine at world size 1: run the multi-GPU step chain anyway (fc_bwd on the forked
    # branch, the bucket all-reduces of the 8-rank plan on the --comm plane, the start-up chain
    # check) - the production ws > 1 chain, rehearsed (and pinned by tests) on one GPU
    force_allreduce: bool = False
    grad_accum: int = 1               # micro-batches per optimizer step (module/CPU path)
    global_loss: bool = False         # log the all-reduced mean loss (module/CPU path, bug B14)
    pg_timeout_s: float | None = None
    model: str = "simplecnn"          # simplecnn | resnet18 (BASELINE config 5)
    image_size: int = 224             # resnet18: synthetic image side
    num_classes: int = 1000           # resnet18
    dataset_size: int = 2048          # resnet18: synthetic images resident per rank
    graph_module: bool = False        # module path on GPU: capture each step in a hipGraph
    dtype: str = "bf16"               # GPU compute precision: bf16 | fp32 (exact fp32 MFMA, reference precision)
    verify_replicas: bool = False     # after every epoch: all ranks' parameters (+ momentum) bitwise equal, or raise
    stall: tuple | None = None        # (epoch, rank, seconds): that rank sleeps before the epoch's first step


def ddp_train(rank: int, world_size: int, epochs: int, batch_size: int,
              opts: TrainOptions | None = None):
    opts = opts or TrainOptions()
    backend = setup(rank=rank, world_size=world_size, backend=opts.backend,
                    timeout_s=opts.pg_timeout_s, device=opts.device)
    # RCCL means the GPU; gloo means the GPU only when it was asked for explicitly (a gloo
    # control plane over GPU tensors + the direct xGMI data plane: same-GPU rehearsals)
    want = (opts.device or os.environ.get("DDP_AMD_DEVICE") or "auto").lower()
    on_gpu = backend == "nccl" or (want == "gpu" and torch.cuda.is_available())
    device = torch.device("cuda", local_rank(rank)) if on_gpu else torch.device("cpu")
    if on_gpu:
        torch.cuda.set_device(device)
    print(f"Rank {rank} initialized", flush=True)
    if opts.grad_accum < 1:
        raise ValueError("--grad_accum must be >= 1")

    if opts.seed is not None:
        torch.manual_seed(opts.seed)  # B15: reproducible init (rank 0's weights win anyway)
    if opts.model == "resnet18":
        if on_gpu and opts.dtype != "bf16":
            raise ValueError("resnet18 on the GPU runs bf16 MFMA kernels only (--dtype bf16)")
        model = resnet18(num_classes=opts.num_classes).to(device)
        if on_gpu and opts.engine == "fused" and rank == 0:
            print("Rank 0: resnet18 runs on the module path (the fused engine is SimpleCNN's)", flush=True)
    elif opts.model == "simplecnn":
        if opts.dtype not in ("bf16", "fp32"):
            raise ValueError(f"--dtype must be bf16 or fp32, got {opts.dtype!r}")
        model = SimpleCNN(compute_dtype=torch.float32 if opts.dtype == "fp32" else torch.bfloat16).to(device)
    else:
        raise ValueError(f"unknown model {opts.model!r}")
    fused = on_gpu and opts.engine == "fused" and opts.model == "simplecnn"
    if fused and (opts.grad_accum != 1 or opts.global_loss):
        raise ValueError("--grad_accum / --global_loss need the module path (--engine module) "
                         "or the CPU path; the fused engine runs one micro-batch per step")
    if fused:
        fs = flat_space(model)

        _verify_and_broadcast(fs, model, world_size)
        ddp_model = model
    else:
        ddp_model = DDP(model, bucket_cap_mb=opts.bucket_cap_mb, comm=module_comm(opts.comm))
        fs = ddp_model.fs
    print(f"Rank {rank} model wrapped in DDP", flush=True)

    if opts.model == "resnet18":
        imgs, labels = synthetic_imagenet(opts.dataset_size, opts.image_size, opts.num_classes)
        loader = DeviceImageLoader(DeviceImages(imgs, labels, device), batch_size, world_size, rank)
        sampler = loader.sampler
    elif on_gpu:
        imgs, labels, src = load_mnist(opts.data_root, opts.data)
        ddata = DeviceMNIST(imgs, labels, device, src)
        loader = DeviceMNISTLoader(ddata, batch_size, world_size, rank)
        sampler = loader.sampler
    else:
        loader, sampler = get_dataloader(batch_size, world_size, rank, root=opts.data_root,
                                         source=opts.data, num_workers=opts.num_workers)
    print(f"Rank {rank}: Dataloader ready", flush=True)
    loss_fn = CrossEntropyLoss()
    opt = FusedSGD(model, lr=opts.lr, momentum=opts.momentum, weight_decay=opts.weight_decay)
    model.train()
    print(f"Rank {rank}: Loss and Optimizer ready", flush=True)

    start_epoch, path = resume(model, opt, opts.checkpoint_dir, rank, world_size,
                               device=device, flat=fs)
    if path is None:
        print(f"Rank {rank}: No checkpoint found, starting from scratch.", flush=True)
    elif rank == 0:
        print(f"Rank {rank}: Resumed from {path}, starting at epoch {start_epoch}", flush=True)

    engine = None
    if fused:
        from .fused_step import EngineOptions, FusedSimpleCNNEngine

        comm = native_comm() if world_size > 1 and dist.get_backend() == "nccl" else None
        force = bool(opts.force_allreduce) and world_size == 1
        if force and comm is None and opts.comm == "rccl" and dist.get_backend() == "nccl":
            comm = native_comm()
        eo = EngineOptions(graph_steps=opts.graph_steps, bucket_cap_mb=opts.bucket_cap_mb,
                           comm=opts.comm, dtype=opts.dtype, force_allreduce=force,
                           plan_world=8 if force else None)
        if opts.fuse_level is not None:
            eo.fuse_level = opts.fuse_level
        engine = FusedSimpleCNNEngine(model, opt, ddata, batch_size, world_size, rank, comm, eo)
        engine.refresh()
        if world_size > 1 or force:
            # the production chain must give the conservative chain's bits across the real
            # peers before training commits to it (VERDICT r3 #3a); else every rank downgrades
            kept = engine.verify_chain()
            if rank == 0:
                print(f"Rank {rank}: start-up chain check "
                      f"{'passed' if kept else 'FAILED -> conservative chain'} ({engine.chain_check})", flush=True)

    for epoch in range(start_epoch, epochs):
        sampler.set_epoch(epoch)
        print(f"Rank {rank}: Starting epoch {epoch}", flush=True)
        t0 = time.perf_counter()

        def log(batch_idx, loss_value):
            if rank == 0:
                print(f"Epoch {epoch} | Batch {batch_idx} | Loss: {loss_value:.4f}", flush=True)

        fault_step = _fault_step(opts.fault, epoch, rank)
        if opts.stall and int(opts.stall[0]) == epoch and int(opts.stall[1]) == rank:
            print(f"Rank {rank}: injected stall of {float(opts.stall[2]):g} s before epoch {epoch}", flush=True)
            time.sleep(float(opts.stall[2]))  # a slow rank: the peers' all-reduces wait for it
        if fused:
            nsteps = engine.run_epoch(epoch, on_loss=log, log_every=opts.log_every,
                                      max_steps=fault_step if fault_step is not None else opts.max_steps)
            engine.synchronize()
        else:
            nsteps = _run_module_epoch(ddp_model, loader, loss_fn, opt, device, log,
                                       opts.log_every,
                                       fault_step if fault_step is not None else opts.max_steps,
                                       opts.grad_accum, opts.global_loss,
                                       graph=on_gpu and opts.graph_module)
        if fault_step is not None:
            _inject_fault(rank, epoch, nsteps)
        if on_gpu:
            torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        _record_metrics(opts, rank, world_size, epoch, nsteps, batch_size, dt,
                        samples_processed(nsteps, batch_size, len(sampler)))

        if opts.verify_replicas and world_size > 1:
            verify_replicas(fs, opt, rank, world_size, epoch)
        if rank == 0 and opts.save:
            save_checkpoint(opts.checkpoint_dir, epoch, model, opt)
        if world_size > 1:
            dist.barrier()  # B13: nobody races past a half-written checkpoint
    cleanup()
    return model


def module_comm(comm: str) -> str:
    """The module path's data plane for the trainer's ``--comm`` (the engine's plan names):
    rccl -> RCCL, xgmi / xgmi1 / xgmi2 / tune -> the direct xGMI kernels, auto -> DDP's own
    choice (RCCL under nccl, xGMI under a gloo control plane)."""
    if comm in ("auto", "rccl"):
        return comm
    if comm in ("xgmi", "xgmi1", "xgmi2", "tune"):
        return "xgmi"
    raise ValueError(f"unknown comm {comm!r}")


def replica_digest(fs, opt) -> str:
    """SHA-1 of this rank's flat parameters (+ momentum): bitwise replica identity."""
    import hashlib

    h = hashlib.sha1(fs.params.detach().cpu().numpy().tobytes())
    mb = getattr(opt, "momentum_buffer", None)
    if mb is not None:
        h.update(mb.detach().cpu().numpy().tobytes())
    return h.hexdigest()


def verify_replicas(fs, opt, rank: int, world_size: int, epoch: int):
    """DDP's invariant, checked: every rank holds bitwise the same parameters and optimizer
    state (a divergence would mean a broken all-reduce or a non-deterministic kernel)."""
    import hashlib

    d = replica_digest(fs, opt)
    allg = [None] * world_size
    dist.all_gather_object(allg, d)
    if any(x != allg[0] for x in allg):
        # which tensors differ (and by how much), for the error message
        per = {n: hashlib.sha1(fs.view(fs.params, n).detach().cpu().numpy().tobytes()).hexdigest()
               for n in fs.names}
        mine = fs.params.detach().cpu()
        allp, allpar = [None] * world_size, [None] * world_size
        dist.all_gather_object(allp, per)
        dist.all_gather_object(allpar, mine)
        bad = [n for n in fs.names if any(p[n] != allp[0][n] for p in allp)]
        worst = max(float((t - allpar[0]).abs().max()) for t in allpar)
        raise RuntimeError(f"epoch {epoch}: replicas diverged across ranks ({allg}); differing tensors "
                           f"{bad}, max |diff| {worst:.3e}")
    if rank == 0:
        print(f"Rank 0: replicas bitwise identical after epoch {epoch} ({d[:12]})", flush=True)


def _fault_step(fault, epoch, rank):
    if not fault:
        return None
    fe, fs_, fr = (list(fault) + [-1])[:3]
    return int(fs_) if int(fe) == epoch and int(fr) in (-1, rank) else None


def _inject_fault(rank, epoch, step):
    """Simulated hard failure: the rank dies without cleanup, as a crash
    would; the launcher tears the job down and a re-run auto-resumes from the last
    checkpoint."""
    print(f"Rank {rank}: injected fault at epoch {epoch} step {step}", flush=True)
    os._exit(17)


def _verify_and_broadcast(fs, model, world_size):
    """DDP construction semantics for the engine path: shape check + rank-0 broadcast."""
    if world_size == 1:
        return
    meta = [(n, fs.shapes[n]) for n in fs.names]
    allm = [None] * world_size
    dist.all_gather_object(allm, meta)
    if any(m != allm[0] for m in allm):
        raise RuntimeError(f"parameter shapes differ across ranks: {allm}")
    with torch.no_grad():
        dist.broadcast(fs.params, src=0)  # one flat collective (SimpleCNN has no buffers)
        fs.params_written()
        bs = buffer_space(model)
        if bs is not None:
            for t in bs.flat_list():  # one flat collective per dtype
                dist.broadcast(t, src=0)


_SYNC_EACH_STEP = os.environ.get("DDP_AMD_SYNC_EACH_STEP") == "1"
_VERIFY_EACH_STEP = os.environ.get("DDP_AMD_VERIFY_EACH_STEP") == "1"


def _verify_step(model, opt, step):
    """Diagnostic (DDP_AMD_VERIFY_EACH_STEP=1): compare the reduced gradients and the
    parameters across ranks after every step; raise at the first difference."""
    import hashlib

    fs = model.fs if hasattr(model, "fs") else flat_space(model)
    torch.cuda.synchronize()
    h = lambda t: hashlib.sha1(t.detach().cpu().numpy().tobytes()).hexdigest()[:10]  # noqa: E731
    mine = {"grads": {n: h(fs.view(fs.grads, n)) for n in fs.names}, "params": h(fs.params)}
    allm = [None] * dist.get_world_size()
    dist.all_gather_object(allm, mine)
    bad = [n for n in fs.names if any(m["grads"][n] != allm[0]["grads"][n] for m in allm)]
    if bad or any(m["params"] != allm[0]["params"] for m in allm):
        raise RuntimeError(f"step {step}: replicas differ - reduced gradients {bad}, params "
                           f"{[m['params'] for m in allm]}")


def _run_module_epoch(model, loader, loss_fn, opt, device, log, log_every, max_steps,
                      grad_accum=1, global_loss=False, graph=False):
    """The reference's loop (train_ddp.py:195-202).  With ``grad_accum`` > 1 the
    optimizer steps every ``grad_accum`` batches; the first ``grad_accum - 1`` backward
    passes run under ``no_sync`` (no all-reduce) and the loss is scaled so the update
    equals one large-batch step.  A ragged tail still flushes with a synchronised
    backward.  ``graph``: full-batch steps replay one captured hipGraph (GraphedStep;
    its capture warm-up steps are real steps on the first batch); a ragged last batch
    runs eagerly."""
    if graph:
        if grad_accum != 1 or global_loss:
            raise ValueError("--graph_module runs one micro-batch per step without loss all-reduce")
        return _run_graphed_epoch(model, loader, loss_fn, opt, log, log_every, max_steps)
    n = 0
    nb = len(loader) if hasattr(loader, "__len__") else None
    if max_steps is not None:
        nb = max_steps if nb is None else min(nb, max_steps)
    opt.zero_grad()
    for batch_idx, batch in enumerate(loader):
        images, labels = batch if isinstance(batch, (tuple, list)) else tuple(batch)
        images = images.to(device, non_blocking=True)
        labels = labels.to(device, non_blocking=True)
        if grad_accum == 1:
            opt.zero_grad()
        last = nb is not None and batch_idx + 1 >= nb
        boundary = grad_accum == 1 or (batch_idx + 1) % grad_accum == 0 or last
        output = model(images)
        loss = loss_fn(output, labels)
        scaled = loss / grad_accum if grad_accum > 1 else loss
        if boundary or not hasattr(model, "no_sync"):
            scaled.backward()
        else:
            with model.no_sync():
                scaled.backward()
        if boundary:
            opt.step()
            if grad_accum > 1:
                opt.zero_grad()
        if _SYNC_EACH_STEP:  # diagnostic: device-synchronise every step
            torch.cuda.synchronize()
        if _VERIFY_EACH_STEP and dist.is_initialized() and dist.get_world_size() > 1:
            _verify_step(model, opt, batch_idx)
        if batch_idx % log_every == 0:
            lv = loss.detach()
            if global_loss and dist.is_initialized() and dist.get_world_size() > 1:
                lv = lv.clone()
                dist.all_reduce(lv)
                lv = lv / dist.get_world_size()
            log(batch_idx, lv.item())
        n += 1
        if max_steps is not None and n >= max_steps:
            break
    return n


class _GraphCache(dict):
    """{input shape: GraphedStep} of one model (a dict subclass so it is weak-referenceable)."""


def _graph_cache(model) -> dict:
    """The model's captured training-step graphs, keyed by input shape.  Kept ON the model
    object (not in a module global keyed by ``id(model)``): it dies with the model, and a
    recycled id can never replay another model's graph."""
    cache = getattr(model, "_ddp_amd_step_graphs", None)
    if cache is None:
        cache = _GraphCache()
        object.__setattr__(model, "_ddp_amd_step_graphs", cache)
    return cache


def _run_graphed_epoch(model, loader, loss_fn, opt, log, log_every, max_steps):
    from .graph_step import GraphedStep

    def step(x, y):
        opt.zero_grad()
        loss = loss_fn(model(x), y)
        loss.backward()
        opt.step()
        return loss

    graphs = _graph_cache(model)
    full = getattr(loader, "batch_size", None)  # the full batch: only that shape is captured
    n = 0
    for batch_idx, (images, labels) in enumerate(loader):
        key = tuple(images.shape)
        if key not in graphs:
            if full is not None and images.shape[0] != full:
                loss = step(images, labels)  # ragged tail: eager, no new capture
            else:
                graphs[key] = GraphedStep(step, (images, labels), warmup=1)  # = this batch's step
                loss = graphs[key].warmup_out
        else:
            loss = graphs[key](images, labels)
        if batch_idx % log_every == 0:
            log(batch_idx, loss.item())
        n += 1
        if max_steps is not None and n >= max_steps:
            break
    return n


def samples_processed(nsteps: int, batch: int, samples_per_rank: int) -> int:
    """Images a rank actually trained on in ``nsteps`` steps of an epoch of
    ``samples_per_rank`` (full batches, then the ragged tail; ``--max_steps`` /
    ``--fault_at`` truncate the epoch)."""
    return min(nsteps * batch, samples_per_rank)


def _record_metrics(opts, rank, ws, epoch, nsteps, batch, dt, samples):
    """``samples``: images this rank processed in the epoch (:func:`samples_processed`)."""
    if not opts.metrics_json or rank != 0:
        return
    import json

    rec = {"epoch": epoch, "world_size": ws, "steps": nsteps, "batch_size": batch,
           "samples_per_rank": samples, "seconds": dt,
           "images_per_sec_aggregate": samples * ws / dt if dt > 0 else None}
    with open(opts.metrics_json, "a") as f:
        f.write(json.dumps(rec) + "\n")
