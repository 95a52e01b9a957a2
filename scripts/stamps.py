"""In-kernel phase timeline of the fused SimpleCNN step (diagnostic).

Runs the headline engine (same construction as bench.py) with the per-TU stamp buffer
set (csrc/kernels/common.h DDP_STAMP), executes a few eager steps, and prints for each
kernel and stamp slot the median / max (over blocks) time since that kernel's first
block started, in microseconds (100 MHz s_memrealtime -> 10 ns resolution).

    python scripts/stamps.py [--batch_size 32] [--fuse_level 1]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

NAMES = {0: "conv3x3_fwd", 1: "fc_bwd", 2: "conv3x3_dgrad", 3: "conv3x3_wgrad",
         4: "grad_reduce", 5: "sgd", 6: "xent", 7: "dgrad-staging", 8: "fwd-dZ2", 9: "xgmi",
         10: "step-head"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch_size", type=int, default=32)
    ap.add_argument("--fuse_level", type=int, default=None)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--graph", action="store_true", help="stamp the last step of a replayed graph")
    ap.add_argument("--dtype", choices=["bf16", "fp32"], default="bf16")
    ap.add_argument("--wgrad_split", type=int, default=None)
    ap.add_argument("--wgrad_rows", type=int, default=None)
    ap.add_argument("--store_a1", type=int, default=None)
    ap.add_argument("--fuse_reduce", type=int, default=None)
    ap.add_argument("--pxt_fwd", type=int, default=None)
    ap.add_argument("--force_allreduce", action="store_true",
                    help="the multi-GPU chain at world size 1 (bucket all-reduces of the 8-rank plan)")
    ap.add_argument("--comm", default="xgmi", help="with --force_allreduce: xgmi | rccl")
    ap.add_argument("--dist_mode", type=int, default=None)
    ap.add_argument("--xgmi_blocks", action="store_true", help="print every xgmi block's stamps")
    ap.add_argument("--head_split", default=None,
                    help="dist_mode 4: 'a,b' - summarise the step head's blocks [0,a) (conv bucket), "
                         "[a,b) (fc bucket) and [b,...) (forward waits) separately")
    ap.add_argument("--min_block", type=int, default=0,
                    help="ignore blocks below this index (dist_mode 4 --graph: the step head's forward "
                         "blocks follow its all-reduce blocks; lower indices hold the graph's first forward)")
    a = ap.parse_args()
    from ddp_amd import native
    from ddp_amd.data import DeviceMNIST, synthetic_mnist
    from ddp_amd.engine import EngineOptions, FusedSimpleCNNEngine
    from ddp_amd.models import SimpleCNN
    from ddp_amd.ops import FusedSGD

    C = native.require()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = SimpleCNN(compute_dtype=torch.float32 if a.dtype == "fp32" else torch.bfloat16).to(dev)
    opt = FusedSGD(model, lr=0.01)
    imgs, labels = synthetic_mnist()
    eo = EngineOptions(use_graph=a.graph, graph_steps=10, dtype=a.dtype)
    comm = None
    if a.force_allreduce:
        import torch.distributed as dist

        from ddp_amd.parallel import free_port, native_comm

        dist.init_process_group("nccl" if a.comm == "rccl" else "gloo", rank=0, world_size=1,
                                init_method=f"tcp://127.0.0.1:{free_port()}",
                                **({"device_id": dev} if a.comm == "rccl" else {}))
        comm = native_comm() if a.comm == "rccl" else None
        eo.force_allreduce, eo.comm, eo.plan_world = True, a.comm, 8
    if a.dist_mode is not None:
        eo.dist_mode = a.dist_mode
    if a.fuse_level is not None:
        eo.fuse_level = a.fuse_level
    for f in ("wgrad_split", "wgrad_rows", "store_a1", "fuse_reduce", "pxt_fwd"):
        if getattr(a, f) is not None:
            setattr(eo, f, getattr(a, f))
    eng = FusedSimpleCNNEngine(model, opt, DeviceMNIST(imgs, labels, dev, "synthetic"),
                               a.batch_size, 1, 0, comm, eo)
    eng.refresh()
    eng.run_steps(10 if a.graph else 3)
    eng.synchronize()
    buf = torch.zeros(C.STAMP_K_COUNT * C.STAMP_KSTRIDE, dtype=torch.int64, device=dev)
    C.stamps_set(buf)
    for _ in range(a.steps):
        buf.zero_()
        torch.cuda.synchronize()
        eng.run_steps(10 if a.graph else 1)
        eng.synchronize()
    C.stamps_set(None)
    st = buf.view(C.STAMP_K_COUNT, 4096, 8).cpu().double()
    t0 = None
    rows = []
    if a.head_split:
        ca, cb = (int(v) for v in a.head_split.split(","))
        hs = st[10]
        t00 = hs[:cb, 0][hs[:cb, 0] > 0].min()
        for name, lo, hi in (("head conv AR", 0, ca), ("head fc AR", ca, cb), ("head fwd", cb, 4096)):
            blk = hs[lo:hi]
            blk = blk[(blk > 0).any(dim=1)]
            parts = []
            for slot in range(8):
                v = blk[:, slot]
                v = v[v > 0]
                if v.numel():
                    d = (v - t00) / 100.0
                    parts.append(f"s{slot} med {d.median().item():6.2f} max {d.max().item():6.2f}")
            print(f"{name:14s} blocks {blk.shape[0]:4d} | " + " ".join(parts))
    for k in range(C.STAMP_K_COUNT):
        s = st[k]
        if a.min_block and NAMES.get(k) in ("conv3x3_fwd", "fwd-dZ2"):
            s = s[a.min_block:]
        live = (s > 0).any(dim=1)  # (step-head forward blocks stamp only their two waits)
        if not live.any():
            continue
        s = s[live]
        kstart = s[:, 0][s[:, 0] > 0].min() if (s[:, 0] > 0).any() else s[s > 0].min()
        t0 = kstart if t0 is None else min(t0, kstart)
        rows.append((kstart, k, s))
    rows.sort(key=lambda r: r[0])
    print(f"batch {a.batch_size}; times in us; 'start' = kernel's first block vs the first kernel")
    for kstart, k, s in rows:
        nb = s.shape[0]
        line = [f"{NAMES.get(k, k):14s} blocks {nb:4d} start {(kstart - t0) / 100:7.2f} |"]
        for slot in range(8):
            v = s[:, slot]
            ok = v > 0
            if not ok.any():
                continue
            d = (v[ok] - kstart) / 100.0
            line.append(f" s{slot} med {d.median().item():6.2f} max {d.max().item():6.2f}")
        if NAMES.get(k) == "xgmi" and a.xgmi_blocks:
            for bi in range(nb):
                vals = " ".join(f"s{sl} {(s[bi, sl] - kstart) / 100.0:6.2f}" for sl in range(8) if s[bi, sl] > 0)
                print(f"    xgmi block {bi:3d}: {vals}")
        # per-block durations (first -> last stamp)
        last = s.max(dim=1).values
        dur = ((last - s[:, 0]) / 100.0)[s[:, 0] > 0]
        line.append(f" | blk dur med {dur.median().item():.2f} max {dur.max().item():.2f}")
        print("".join(line))


if __name__ == "__main__":
    main()
