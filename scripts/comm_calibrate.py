"""Fit the xGMI all-reduce cost model (parallel/comm_calibration.py) on N ranks.

    python scripts/comm_calibrate.py --ranks 2 [--out gpurun_out/cal.json]

Spawns N processes (gloo bootstrap, one GPU per rank when there are enough GPUs, else all
on cuda:0 - a same-GPU rehearsal), sweeps the two-shot and one-shot bucket kernels over
bucket sizes, fits launch / barrier / link efficiency and stores the fit with its
provenance (topology "xgmi" or "same-gpu", world size, device, date) in --out.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def worker(rank, world, port, out, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        ngpu = torch.cuda.device_count()
        torch.cuda.set_device(rank % max(1, ngpu))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from ddp_amd.parallel import comm_calibration as cc

        fit = cc.calibrate(rank, world, torch.device("cuda", torch.cuda.current_device()))
        topo = cc.topology(world, rank=rank)
        if rank == 0 and fit is not None:
            rec = cc.save(fit, world, topo, path=out)
            print(json.dumps(rec), flush=True)
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok" if fit is not None else "no xgmi"))
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=2)
    ap.add_argument("--out", default="gpurun_out/xgmi_calibration.json")
    a = ap.parse_args()
    from ddp_amd.parallel import free_port

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=worker, args=(r, a.ranks, port, a.out, q)) for r in range(a.ranks)]
    for p in ps:
        p.start()
    res = [q.get(timeout=300) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    print(res)
    sys.exit(0 if all(r[1] == "ok" for r in res) else 1)


if __name__ == "__main__":
    main()
