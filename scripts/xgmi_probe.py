"""Multi-process (one GPU) probe of the xGMI all-reduce: world size, timing, errors."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, torch.distributed as dist
import torch.multiprocessing as mp


def worker(rank, world, port, timeout):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ddp_amd import native
    C = native.require()
    store = dist.distributed_c10d._get_default_store()
    grads = torch.ones(520586, device="cuda") * (rank + 1)
    x = C.XgmiComm(rank, world, 0)
    x.add_channel(0, 501770); x.add_channel(501770, 18816)
    x.set_data(grads)
    x.set_timeout(timeout)
    store.set(f"h/{rank}", x.export_handles())
    x.import_handles([store.get(f"h/{r}") for r in range(world)])
    dist.barrier()
    for it in range(20):
        t0 = time.perf_counter()
        x.all_reduce(0); x.all_reduce(1)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if it < 3 or it == 19:
            print(f"[{rank}] it {it} {dt*1e6:.0f} us err={x.error_flags()} v={grads[0].item()} {grads[-1].item()}", flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    world = int(sys.argv[1]); timeout = float(sys.argv[2])
    from ddp_amd.parallel import free_port
    mp.spawn(worker, args=(world, free_port(), timeout), nprocs=world)
