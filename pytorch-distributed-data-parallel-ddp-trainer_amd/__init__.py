"""ddp_amd - an MI355X-native (gfx950 / CDNA4) data-parallel training framework.

Same capabilities and CLI as zahmedy/PyTorch-Distributed-Data-Parallel-DDP-Trainer
(SimpleCNN on MNIST, DistributedSampler sharding, rank-0 per-epoch checkpoints,
auto-resume), built MI355X-first: hand-written HIP/MFMA kernels for the whole
training step, a native RCCL communicator + bucketed gradient reducer, and a
hipGraph-captured fused step engine.

Subpackages: ``models`` (SimpleCNN, native-layout layers), ``ops`` (HIP autograd
Functions, fused SGD, PyTorch references), ``parallel`` (process groups, launcher,
DDP + reducer, RCCL comm), ``data`` (MNIST-shaped data, sampler, device loader),
``engine`` (trainer + fused graph-captured step), ``utils`` (checkpoint, logging,
timing, debug).  Import name ``ddp_amd`` (symlink to this directory).
"""
__version__ = "0.1.0"
