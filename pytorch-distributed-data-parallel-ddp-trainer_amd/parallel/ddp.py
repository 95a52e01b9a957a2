"""DistributedDataParallel for the module path (reference train_ddp.py:34 ``DDP(model)``).

Behaviour kept from the reference's DDP:

* construction: verify parameter shapes across ranks, then broadcast rank 0's
  parameters (ONE collective over the flat parameter buffer) and buffers;
* gradient buckets in gradient-ready order with torch's size rule (first bucket
  1 MiB, then ``bucket_cap_mb``) - for SimpleCNN this reproduces the reference's
  rebuilt buckets ``[fl.bias, fl.weight]`` and ``[net.2.*, net.0.*]``;
* a bucket is all-reduced as soon as its last gradient is accumulated (overlap
  with the rest of backward); ``loss.backward()`` returns with averaged
  gradients (sum_r g_r / ws);
* ``broadcast_buffers``: rank 0's buffers are broadcast before each forward - ONE
  collective over a flat byte buffer that every module buffer is a view into
  (``BufferSpace``; torch coalesces the same way), stream-ordered RCCL from our native
  communicator on the GPU, so the whole step stays hipGraph-capturable at any world size;
* ``no_sync()`` for gradient accumulation; ``.module`` for the wrapped model.

MI355X-first differences: parameters and gradients live in one flat fp32 buffer
each (``FlatSpace``), so buckets are plain slices (no pack / unpack copies,
``gradient_as_bucket_view`` always on).  On GPUs the bucket all-reduces are
issued by the native C++ reducer (``csrc/runtime/reducer.cpp``) on its own HIP
stream through our RCCL communicator (a pre-multiplied SUM: every rank's bucket times
1/ws inside the reduction, ``Comm::all_reduce_premul``) or the direct xGMI kernels (1/ws
in their publish pass, fixed rank-order SUM); on CPU/gloo a Python reducer
with async c10d work handles implements the same protocol.
"""
from __future__ import annotations

import contextlib

import torch
import torch.distributed as dist
import torch.nn as nn

from ..models.layers import FlatSpace, buffer_space, flat_space


def bucket_plan(fs: FlatSpace, bucket_cap_mb: float = 25.0, first_bucket_mb: float = 1.0):
    """Bucket assignment over the flat (gradient-ready) order: list of lists of names."""
    buckets, cur, size = [], [], 0
    limit = int(first_bucket_mb * 1024 * 1024)
    for n in fs.names:
        cur.append(n)
        size += fs.numels[n] * 4
        if size >= limit:
            buckets.append(cur)
            cur, size = [], 0
            limit = int(bucket_cap_mb * 1024 * 1024)
    if cur:
        buckets.append(cur)
    return buckets


def check_plan(fs: FlatSpace, buckets):
    """An explicit bucket plan must cover every parameter once, in gradient-ready order."""
    flat = [n for b in buckets for n in b]
    if flat != list(fs.names) or any(not b for b in buckets):
        raise ValueError("bucket plan must split the gradient-ready parameter order into non-empty "
                         f"contiguous buckets: got {[len(b) for b in buckets]} over {len(fs.names)} params")
    return [list(b) for b in buckets]


def bucket_ranges(fs: FlatSpace, buckets):
    """(offset, numel) of each bucket in the flat buffer (contiguous by construction)."""
    out = []
    for i, b in enumerate(buckets):
        start = fs.offsets[b[0]]
        end = fs.offsets[buckets[i + 1][0]] if i + 1 < len(buckets) else fs.numel
        out.append((start, end - start))
    return out


class _PyReducer:
    """c10d reducer (gloo / any backend): prescale by 1/ws, async SUM all-reduce per bucket."""

    def __init__(self, fs: FlatSpace, ranges, pg=None):
        self.fs, self.ranges, self.pg = fs, ranges, pg
        self.ws = dist.get_world_size(pg)
        self.works = {}

    def launch(self, b):
        off, n = self.ranges[b]
        view = self.fs.grads[off:off + n]
        if self.ws > 1:
            view.mul_(1.0 / self.ws)
            self.works[b] = dist.all_reduce(view, op=dist.ReduceOp.SUM, group=self.pg, async_op=True)

    def finalize(self):
        for w in self.works.values():
            w.wait()
        self.works.clear()


class _NativeReducer:
    """Native C++ reducer (GPU): per-bucket all-reduce (mean) on a dedicated HIP stream -
    RCCL, or the direct xGMI kernels (``comm="xgmi"``: fixed rank-order sums, bitwise
    identical on every rank; the only data plane when the ranks bootstrapped over gloo)."""

    def __init__(self, fs: FlatSpace, buckets, ranges, comm: str = "rccl"):
        from .. import native
        from .process_group import native_comm

        C = native.require()
        names = fs.names
        pb = {n: i for i, b in enumerate(buckets) for n in b}
        rccl = dist.get_backend() == "nccl"
        self.kind = "rccl"
        self.xgmi = None
        if comm == "xgmi":
            from .xgmi import MODULE_GRID_CAP, channel_plan, create_xgmi

            from .bucket_model import XgmiCost

            # small buckets: the one-shot kernel (one cross-GPU barrier), below the cost
            # model's crossover for this world size and the one-grid cap the engine uses
            # (bucket_model.ONESHOT_MAX_ELEMS: each one-shot channel also holds 2 x its bucket
            # of stage memory - uncapped, every ResNet-18 bucket got one at N <= 2, ~94 MB more)
            lim = XgmiCost.calibrated(dist.get_world_size()).oneshot_cap_elems()
            oneshot = tuple(b for b, (_, n) in enumerate(ranges) if n <= lim)
            # the bucket kernels run next to the backward: small spinning grid
            self.xgmi = create_xgmi(fs.grads, ranges, dist.get_rank(), dist.get_world_size(),
                                    oneshot=oneshot, grid_cap=MODULE_GRID_CAP)
            if self.xgmi is None and not rccl:
                raise RuntimeError("xGMI self-test failed and the gloo group has no RCCL plane")
            if self.xgmi is not None:
                cp = channel_plan(len(ranges), oneshot)
                self.channels = [cp[(b, b in oneshot)] for b in range(len(ranges))]
                self.kind = "xgmi"
        self.r = C.Reducer(native_comm() if rccl else None, fs.grads, [fs.offsets[n] for n in names],
                           [fs.numels[n] for n in names], [pb[n] for n in names],
                           [o for o, _ in ranges], [n for _, n in ranges], False)
        if self.xgmi is not None:
            self.r.set_xgmi(self.xgmi, self.channels)
        self.index = {n: i for i, n in enumerate(names)}

    def mark_ready(self, name):
        self.r.mark_ready(self.index[name], None)

    def finalize(self):
        self.r.finalize()


class DistributedDataParallel(nn.Module):
    def __init__(self, module: nn.Module, device_ids=None, output_device=None,
                 broadcast_buffers: bool = True, bucket_cap_mb: float = 25.0,
                 find_unused_parameters: bool = False, process_group=None,
                 first_bucket_mb: float = 1.0, native: bool | None = None, comm: str = "auto",
                 buckets: list | None = None):
        """``comm`` (GPU, default group): ``"rccl"``, ``"xgmi"`` (the direct kernels) or
        ``"auto"`` - RCCL under the nccl backend, xGMI when the ranks bootstrapped over gloo
        (several ranks on one GPU rehearse the multi-GPU path that way).  ``buckets``: an
        explicit plan (lists of parameter names covering the gradient-ready order, e.g.
        ``bucket_model.module_plan``) instead of torch's size rule."""
        super().__init__()
        self.module = module
        self.process_group = process_group
        self.broadcast_buffers = broadcast_buffers
        self.find_unused_parameters = find_unused_parameters
        self.fs = flat_space(module)
        self.bufs = buffer_space(module)
        self.world_size = dist.get_world_size(process_group)
        self.rank = dist.get_rank(process_group)
        # global rank of the group's rank 0: the source of every DDP broadcast
        self._src = dist.get_global_rank(process_group, 0) if process_group is not None else 0
        self.buffer_broadcasts = 0
        self._verify_params()
        self._sync_module_states()
        self.buckets = (check_plan(self.fs, buckets) if buckets is not None
                        else bucket_plan(self.fs, bucket_cap_mb, first_bucket_mb))
        self.ranges = bucket_ranges(self.fs, self.buckets)
        self._bucket_of = {n: i for i, b in enumerate(self.buckets) for n in b}
        self._pending = [len(b) for b in self.buckets]
        use_native = native if native is not None else (self.fs.params.is_cuda and process_group is None)
        if comm not in ("auto", "rccl", "xgmi"):
            raise ValueError(f"comm must be auto|rccl|xgmi, got {comm!r}")
        if comm == "auto":
            comm = "rccl" if dist.get_backend(process_group) == "nccl" else "xgmi"
        if use_native and comm == "rccl" and dist.get_backend(process_group) != "nccl":
            raise ValueError("comm='rccl' needs the nccl (RCCL) backend")
        if use_native and self.world_size == 1:
            comm = "rccl" if dist.get_backend(process_group) == "nccl" else "none"
        self._native = None
        if use_native and comm != "none":
            self._native = _NativeReducer(self.fs, self.buckets, self.ranges, comm)
        elif use_native and comm == "none":
            use_native = False  # world size 1 over gloo: nothing to reduce
        self.comm_kind = self._native.kind if self._native is not None else "c10d"
        self._py = None if use_native else _PyReducer(self.fs, self.ranges, process_group)
        self._sync_enabled = True
        self._queued = False
        self._launched = [False] * len(self.buckets)
        self._hooks = []
        for n in self.fs.names:
            p = self.fs.param(n)
            if p.requires_grad:
                # also fires for gradients the HIP Functions wrote in place (ops/direct_grad.py)
                self._hooks.append(p.register_post_accumulate_grad_hook(self._make_hook(n)))
        self.allreduce_buckets_launched = 0
        self._stream = torch.cuda.current_stream(self.fs.params.device) if self.fs.params.is_cuda else None

    # ---------------------------------------------------------------- construction sync
    def _verify_params(self):
        meta = [(n, self.fs.shapes[n]) for n in self.fs.names]
        allm = [None] * self.world_size
        dist.all_gather_object(allm, meta, group=self.process_group)
        for r, m in enumerate(allm):
            if m != allm[0]:
                raise RuntimeError(f"DDP: rank {r} parameters {m} differ from rank 0 {allm[0]}")

    @torch.no_grad()
    def _sync_module_states(self):
        if self.world_size == 1:
            return
        self._broadcast(self.fs.params)
        self.fs.params_written()  # stale bf16 weight copies otherwise (no version bump)
        if self.bufs is not None:
            for t in self.bufs.flat_list():  # one per dtype
                self._broadcast(t)

    def _broadcast(self, t: torch.Tensor):
        """One broadcast of a flat buffer from the group's rank 0: our native RCCL
        communicator on the current HIP stream (graph-capturable) for device tensors in the
        default group, c10d otherwise."""
        if t.is_cuda and self.process_group is None and dist.get_backend() == "nccl":
            from .process_group import native_comm

            native_comm().broadcast(t, self._src, 0)
        else:
            dist.broadcast(t, src=self._src, group=self.process_group)

    # ---------------------------------------------------------------- hooks
    def _make_hook(self, name):
        def hook(p):
            if not self._sync_enabled:
                return
            view = self.fs.view(self.fs.grads, name)
            if p.grad is not None and p.grad.data_ptr() != view.data_ptr():
                view.copy_(p.grad)  # someone replaced .grad (set_to_none); re-home it
                p.grad = view
            if not self._queued:
                self._queued = True
                torch.autograd.Variable._execution_engine.queue_callback(self._finalize)
            b = self._bucket_of[name]
            if self._native is not None:
                # the forward's stream, not the hook's: autograd may run AccumulateGrad
                # hooks with another current stream (a leaf's stream), which under hipGraph
                # capture would leave the bucket all-reduce outside the captured graph
                with torch.cuda.stream(self._stream):
                    self._native.mark_ready(name)
            self._pending[b] -= 1
            if self._pending[b] == 0:
                self._launched[b] = True
                self.allreduce_buckets_launched += 1
                if self._py is not None:
                    self._py.launch(b)
        return hook

    def _finalize(self):
        if self._native is not None:
            with torch.cuda.stream(self._stream):
                self._native.finalize()
        else:
            for b, done in enumerate(self._launched):
                if not done:
                    self._py.launch(b)
            self._py.finalize()
        self._pending = [len(b) for b in self.buckets]
        self._launched = [False] * len(self.buckets)
        self._queued = False

    # ---------------------------------------------------------------- API
    @contextlib.contextmanager
    def no_sync(self):
        old = self._sync_enabled
        self._sync_enabled = False
        try:
            yield
        finally:
            self._sync_enabled = old

    def forward(self, *args, **kwargs):
        if self.fs.params.is_cuda:
            # the step's compute stream: the bucket all-reduces order after it (see the hooks)
            self._stream = torch.cuda.current_stream(self.fs.params.device)
        if self.broadcast_buffers and self.world_size > 1 and self.bufs is not None:
            self.bufs = buffer_space(self.module)  # rehomed (or rebuilt after a .to())
            with torch.no_grad():
                for t in self.bufs.flat_list():  # one per dtype
                    self._broadcast(t)
            self.buffer_broadcasts += 1
        return self.module(*args, **kwargs)


DDP = DistributedDataParallel
