"""Diagnostic: does a graph-captured native Reducer bucket all-reduce (xGMI, 2 ranks on one
GPU, gloo bootstrap) reduce on replay?  Prints per-case max errors."""
import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def worker(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ddp_amd import native
    from ddp_amd.parallel.xgmi import create_xgmi

    C = native.require()
    n = 1 << 16
    grads = torch.zeros(2 * n, device="cuda")
    ranges = [(0, n), (n, n)]
    x = create_xgmi(grads, ranges, rank, world)
    r = C.Reducer(None, grads, [0, n], [n, n], [0, 1], [0, n], [n, n], False)
    r.set_xgmi(x, [0, 1])
    src = torch.full((2 * n,), float(rank + 1), device="cuda")

    def step():
        grads.copy_(src)
        r.mark_ready(0, None)
        r.mark_ready(1, None)
        r.finalize()
        out.copy_(grads)

    out = torch.zeros_like(grads)
    step()
    torch.cuda.synchronize()
    print(f"rank {rank} eager: {out[:2].tolist()} {out[-2:].tolist()}", flush=True)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        step()
    torch.cuda.synchronize()
    dist.barrier()
    out.zero_()
    src.fill_(float(10 * (rank + 1)))
    g.replay()
    torch.cuda.synchronize()
    print(f"rank {rank} replay: {out[:2].tolist()} {out[-2:].tolist()} flags {x.error_flags()}", flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    from ddp_amd.parallel import free_port

    mp.start_processes(worker, args=(2, free_port()), nprocs=2, start_method="spawn")
