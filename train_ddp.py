"""DDP trainer CLI - drop-in for the reference's ``train_ddp.py``.

    python train_ddp.py [--epochs 10] [--batch_size 32] [--world_size N]
    torchrun --nproc_per_node=N train_ddp.py --epochs 3 --batch_size 64

Same flags and defaults as the reference (train_ddp.py:215-219: ``--epochs``
10, per-rank ``--batch_size`` 32) plus the README's documented ``--world_size``
(reference bug B1) and MI355X options.  Under torchrun the ranks come from the
environment (no nested spawn, bug B3); otherwise ``--world_size`` processes are
spawned (default: all visible GPUs, or 2 on a CPU host).  Checkpoints go to
``./checkpoints/epoch_{N}.pt`` and a re-run resumes from the newest one.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from ddp_amd.engine.trainer import TrainOptions, ddp_train  # noqa: E402
from ddp_amd.parallel.launcher import launch  # noqa: E402


def parse_args(argv=None):
    p = argparse.ArgumentParser(description="DDP Training Script (MI355X-native)")
    p.add_argument("--epochs", type=int, default=10, help="Number of training epochs")
    p.add_argument("--batch_size", type=int, default=32, help="Batch size for training (per rank)")
    p.add_argument("--world_size", type=int, default=None,
                   help="processes to spawn when not under torchrun (default: #GPUs, or 2 on CPU)")
    p.add_argument("--backend", choices=["rccl", "nccl", "gloo"], default=None,
                   help="collective backend (default: rccl on GPU, gloo on CPU)")
    p.add_argument("--device", choices=["auto", "gpu", "cpu"], default="auto",
                   help="gpu: fail unless a HIP device is usable; cpu: gloo plumbing run; auto: the GPU "
                        "when usable, CPU only on a host without one (never a silent fallback on a GPU host)")
    p.add_argument("--dtype", choices=["bf16", "fp32"], default="bf16",
                   help="GPU compute precision: bf16 MFMA operands (fp32 masters/grads/optimizer) or "
                        "exact fp32 MFMA (the reference's fp32 nn.Conv2d/nn.Linear precision)")
    p.add_argument("--engine", choices=["fused", "module"], default="fused",
                   help="GPU step: fused native engine (hipGraph) or module path (autograd)")
    p.add_argument("--data", choices=["auto", "mnist", "synthetic"], default="auto",
                   help="MNIST IDX files under --data_root if present, else synthetic MNIST-shaped")
    p.add_argument("--data_root", default="./data")
    p.add_argument("--checkpoint_dir", default="./checkpoints")
    p.add_argument("--no_save", action="store_true", help="do not write checkpoints")
    p.add_argument("--lr", type=float, default=0.01)
    p.add_argument("--momentum", type=float, default=0.0)
    p.add_argument("--weight_decay", type=float, default=0.0)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--log_every", type=int, default=100)
    p.add_argument("--graph_steps", type=int, default=100, help="steps per captured hipGraph")
    p.add_argument("--bucket_cap_mb", type=float, default=25.0)
    p.add_argument("--num_workers", type=int, default=2, help="CPU DataLoader workers")
    p.add_argument("--max_steps", type=int, default=None, help="cap steps per epoch (module/CPU path)")
    p.add_argument("--metrics_json", default=None, help="append per-epoch img/s records (rank 0)")
    p.add_argument("--fuse_level", type=int, default=None, choices=[0, 1, 3],
                   help="fused engine: 0 = a1 materialised, separate conv1/xent/dgrad/wgrad/SGD kernels; "
                        "1 = 3 kernels/step; 3 = dZ2 in the forward, fc weight gradient inside the conv "
                        "backward: 2 kernels/step (default)")
    p.add_argument("--comm", choices=["auto", "tune", "xgmi", "xgmi1", "xgmi2", "rccl"], default="auto",
                   help="bucket all-reduce data plane at world size > 1. Fused engine: auto = the direct xGMI "
                        "kernels (one-shot for the small bucket; RCCL if their self-test fails) - deterministic, "
                        "so resumes reduce in the same order; tune = fastest of xgmi2 / xgmi1 / RCCL on the "
                        "node. Module path (--engine module, resnet18): rccl, or xgmi for any xgmi* / tune; "
                        "auto = RCCL under the rccl backend, xGMI under gloo")
    p.add_argument("--grad_accum", type=int, default=1,
                   help="micro-batches per optimizer step (module/CPU path; DDP no_sync)")
    p.add_argument("--global_loss", action="store_true",
                   help="log the all-reduced mean loss instead of rank 0's local loss (module/CPU path)")
    p.add_argument("--pg_timeout_min", type=float, default=30.0,
                   help="process-group timeout in minutes (reference default 30)")
    p.add_argument("--model", choices=["simplecnn", "resnet18"], default="simplecnn",
                   help="resnet18 = BASELINE config 5 on synthetic ImageNet-shaped data (module path)")
    p.add_argument("--image_size", type=int, default=224, help="resnet18: synthetic image side")
    p.add_argument("--num_classes", type=int, default=1000, help="resnet18: classes")
    p.add_argument("--dataset_size", type=int, default=2048, help="resnet18: synthetic images")
    p.add_argument("--graph_module", action="store_true",
                   help="module path on GPU: replay each training step as one captured hipGraph")
    p.add_argument("--fault_at", default=None, metavar="EPOCH:STEP[:RANK]",
                   help="simulate a crash (os._exit) at that step; re-run to auto-resume")
    p.add_argument("--stall_at", default=None, metavar="EPOCH:RANK:SECONDS",
                   help="simulate a slow rank: it sleeps before that epoch's first step")
    p.add_argument("--force_allreduce", action="store_true",
                   help="rehearsal on one GPU: run the multi-GPU fused step chain at world size 1 (forked "
                        "fc branch, bucket all-reduces of the 8-rank plan on the --comm plane, chain check)")
    p.add_argument("--verify_replicas", action="store_true",
                   help="after every epoch check that all ranks' parameters and momentum are bitwise equal")
    return p.parse_args(argv)


def main(argv=None):
    a = parse_args(argv)
    opts = TrainOptions(lr=a.lr, momentum=a.momentum, weight_decay=a.weight_decay,
                        backend=a.backend, device=a.device, engine=a.engine, dtype=a.dtype, data=a.data, data_root=a.data_root,
                        checkpoint_dir=a.checkpoint_dir, save=not a.no_save, seed=a.seed,
                        log_every=a.log_every, graph_steps=a.graph_steps,
                        bucket_cap_mb=a.bucket_cap_mb, num_workers=a.num_workers,
                        max_steps=a.max_steps, metrics_json=a.metrics_json,
                        fuse_level=a.fuse_level, grad_accum=a.grad_accum,
                        global_loss=a.global_loss, pg_timeout_s=a.pg_timeout_min * 60.0,
                        comm=a.comm, model=a.model, image_size=a.image_size,
                        num_classes=a.num_classes, dataset_size=a.dataset_size,
                        graph_module=a.graph_module, verify_replicas=a.verify_replicas,
                        force_allreduce=a.force_allreduce,
                        stall=tuple(float(v) for v in a.stall_at.split(":")) if a.stall_at else None,
                        fault=tuple(int(v) for v in a.fault_at.split(":")) if a.fault_at else None)
    launch(ddp_train, a.world_size, args=(a.epochs, a.batch_size, opts))


if __name__ == "__main__":
    main()
