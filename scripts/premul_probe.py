"""RCCL pre-multiplied SUM at world size 1: which sizes come out right (diagnostic).

    python scripts/premul_probe.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    from ddp_amd.parallel import free_port, native_comm

    dist.init_process_group("nccl", rank=0, world_size=1, init_method=f"tcp://127.0.0.1:{free_port()}",
                            device_id=torch.device("cuda", 0))
    comm = native_comm()
    for s in (0.5, 1.0 / 3.0):
        for n in (4, 63, 64, 1000, 1024, 4096, 65536, 100003, 262144, 1 << 20, 4 << 20):
            x = torch.randn(n, device="cuda")
            want = x * torch.tensor(s, dtype=torch.float32, device="cuda")
            y = x.clone()
            comm.all_reduce_premul(y, s)
            torch.cuda.synchronize()
            bad = (y != want).nonzero().flatten()
            unscaled = int((y == x).sum()) if s != 1.0 else 0
            print(f"scale {s:.4f} n {n:8d}: mismatches {bad.numel():8d} first {int(bad[0]) if bad.numel() else -1:8d} "
                  f"unscaled {unscaled}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
