"""Probe: can 2 RCCL ranks share one GPU on this box?  Exercises the native Comm and the
fused engine at world_size=2 (both ranks on cuda:0) if RCCL allows it."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, torch.distributed as dist
rank, ws = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
from ddp_amd.parallel import setup, native_comm
os.environ["LOCAL_RANK"] = "0"
setup(rank, ws, backend="nccl", verbose=False)
print(f"[{rank}] pg ok", flush=True)
c = native_comm()
t = torch.full((1024,), float(rank + 1), device="cuda")
c.all_reduce(t, 0, 0); torch.cuda.synchronize()
print(f"[{rank}] native allreduce -> {t[0].item()} (expect {ws*(ws+1)/2})", flush=True)
from ddp_amd.data import DeviceMNIST, synthetic_mnist
from ddp_amd.engine import EngineOptions, FusedSimpleCNNEngine
from ddp_amd.models import SimpleCNN
from ddp_amd.models.layers import flat_space
from ddp_amd.ops import FusedSGD
torch.manual_seed(rank)
m = SimpleCNN().cuda(); fs = flat_space(m)
dist.broadcast(fs.params, src=0)
opt = FusedSGD(m, lr=0.01)
imgs, labels = synthetic_mnist(4096)
eng = FusedSimpleCNNEngine(m, opt, DeviceMNIST(imgs, labels, torch.device("cuda", 0)), 32, ws, rank, c,
                           EngineOptions(graph_steps=5))
eng.refresh()
eng.run_steps(12); eng.synchronize()
d = fs.params.double().sum().item()
ds = [None] * ws; dist.all_gather_object(ds, d)
print(f"[{rank}] engine ws={ws} params checksum {d:.6f} all-equal={len(set(ds)) == 1}", flush=True)
dist.destroy_process_group()
