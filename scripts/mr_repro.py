"""2 ranks, ONE GPU, gloo control plane: SimpleCNN module path + our DDP over the xGMI data
plane; compare parameters across ranks after every step (diagnostic for replica divergence).

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 scripts/mr_repro.py [--sync]
"""
import argparse
import hashlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sync", action="store_true", help="device-synchronise after every backward")
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--check_grads", action="store_true", help="hash the reduced gradients each step (syncs!)")
    ap.add_argument("--oneshot_max", default=None)
    ap.add_argument("--sync_step", action="store_true", help="device-synchronise after opt.step")
    ap.add_argument("--sync_fwd", action="store_true", help="device-synchronise after the forward")
    a = ap.parse_args()
    if a.oneshot_max:
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
    opt = FusedSGD(m, lr=0.01)
    lossf = CrossEntropyLoss()
    g = torch.Generator(device="cuda").manual_seed(rank)
    first_bad = None
    for it in range(a.steps):
        x = torch.rand(32, 1, 28, 28, device="cuda", generator=g)
        y = torch.randint(0, 10, (32,), device="cuda", generator=g)
        opt.zero_grad()
        out = ddp(x)
        if a.sync_fwd:
            torch.cuda.synchronize()
        lossf(out, y).backward()
        if a.sync:
            torch.cuda.synchronize()
        gd = {n: hashlib.sha1(ddp.fs.view(ddp.fs.grads, n).cpu().numpy().tobytes()).hexdigest()[:8]
              for n in ddp.fs.names} if a.check_grads else {}
        opt.step()
        if a.sync_step:
            torch.cuda.synchronize()
        allg = [None] * ws
        dist.all_gather_object(allg, gd)
        pd = hashlib.sha1(ddp.fs.params.detach().cpu().numpy().tobytes()).hexdigest()[:8]
        allp = [None] * ws
        dist.all_gather_object(allp, pd)
        bad = [n for n in gd if allg[0][n] != allg[1][n]] + (["params"] if allp[0] != allp[1] else [])
        if bad and first_bad is None:
            first_bad = (it, bad)
    if rank == 0:
        print(f"kind={ddp.comm_kind} sync={a.sync} first divergent step / grads: {first_bad}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
