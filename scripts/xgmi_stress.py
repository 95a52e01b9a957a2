"""xGMI all-reduce stress on ONE GPU shared by 2 ranks (gloo control plane): every step
computes each rank's LOCAL SimpleCNN gradient (no_sync), then the DDP-reduced one, and
checks the reduced gradient against the exact fixed-order mean (L0 + L1) * 0.5 on both
ranks.  On a mismatch it reports the rank, element count, the first bad flat indices
and whether the bad value looks like a stale / missing peer contribution; parameters
are re-synchronised from rank 0 so the run keeps counting.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
        scripts/xgmi_stress.py --steps 200 [--oneshot_max 0]
"""
import argparse
import time
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--oneshot_max", default=None)
    a = ap.parse_args()
    if a.oneshot_max is not None:
        os.environ["DDP_AMD_XGMI_ONESHOT_MAX"] = a.oneshot_max
    rank, ws = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    from ddp_amd.models import SimpleCNN
    from ddp_amd.ops import CrossEntropyLoss, FusedSGD
    from ddp_amd.parallel import DistributedDataParallel

    torch.manual_seed(0)
    m = SimpleCNN().cuda()
    ddp = DistributedDataParallel(m, comm="xgmi")
    fs = ddp.fs
    opt = FusedSGD(m, lr=0.01)
    lossf = CrossEntropyLoss()
    g = torch.Generator(device="cuda").manual_seed(rank)
    bad_steps, reports, first_err = 0, [], None
    t0 = time.perf_counter()
    for it in range(a.steps):
        x = torch.rand(32, 1, 28, 28, device="cuda", generator=g)
        y = torch.randint(0, 10, (32,), device="cuda", generator=g)
        opt.zero_grad()
        with ddp.no_sync():
            lossf(ddp(x), y).backward()
        local = fs.grads.clone()
        opt.zero_grad()
        ts = time.perf_counter()
        lossf(ddp(x), y).backward()
        torch.cuda.synchronize()
        if it < 3:
            reports.append(f"rank {rank} step {it}: synced backward took {time.perf_counter() - ts:.3f} s")
        red = fs.grads.detach().cpu()
        allloc = [torch.zeros_like(red) for _ in range(ws)]
        dist.all_gather(allloc, local.cpu())
        exp = allloc[0].clone()
        for p in range(1, ws):
            exp += allloc[p]
        exp *= 1.0 / ws
        err = ddp._native.xgmi.error_flags() if ddp._native is not None and ddp._native.xgmi is not None else 0
        if err and first_err is None:
            from ddp_amd.parallel.xgmi import describe_xgmi_error
            first_err = (it, describe_xgmi_error(err), round(time.perf_counter() - t0, 2))
        badm = red != exp
        nb = torch.tensor([int(badm.sum())])
        dist.all_reduce(nb)
        if int(nb) > 0:
            bad_steps += 1
            if badm.any() and len(reports) < 9:
                idx = badm.nonzero().flatten()
                i0 = int(idx[0])
                own = allloc[rank][i0] * (1.0 / ws)
                names = sorted({n for n in fs.names
                                for i in idx[:2000].tolist()
                                if fs.offsets[n] <= i < fs.offsets[n] + fs.numels[n]})
                reports.append(f"step {it} rank {rank}: {idx.numel()} bad elems in {names}, first {idx[:6].tolist()} "
                               f"span [{int(idx[0])},{int(idx[-1])}] got {float(red[i0]):.6g} exp {float(exp[i0]):.6g} "
                               f"own/ws {float(own):.6g}")
        opt.step()
        with torch.no_grad():  # re-synchronise the replicas
            p = fs.params.cpu()
            dist.broadcast(p, 0)
            fs.params.copy_(p)
            fs.params_written()
    allr = [None] * ws
    dist.all_gather_object(allr, reports + [f"rank {rank}: first xGMI error {first_err}, {time.perf_counter() - t0:.1f} s"])
    if rank == 0:
        print(f"kind={ddp.comm_kind} oneshot_max={a.oneshot_max} steps={a.steps} bad_steps={bad_steps}", flush=True)
        for r in allr:
            for line in r:
                print("  " + line, flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
