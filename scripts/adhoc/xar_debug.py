import os, sys
sys.path.insert(0, os.getcwd())
os.environ["DDP_AMD_XAR_DEBUG"] = "1"
import torch
import torch.distributed as dist
from ddp_amd.data import DeviceMNIST, synthetic_mnist
from ddp_amd.engine import EngineOptions, FusedSimpleCNNEngine
from ddp_amd.models import SimpleCNN
from ddp_amd.ops import FusedSGD
from ddp_amd.parallel import free_port
dist.init_process_group("gloo", rank=0, world_size=1, init_method=f"tcp://127.0.0.1:{free_port()}")
dev = torch.device("cuda", 0)
imgs, labels = synthetic_mnist(2048)
data = DeviceMNIST(imgs, labels, dev)
torch.manual_seed(0)
m = SimpleCNN().to(dev)
e = FusedSimpleCNNEngine(m, FusedSGD(m, lr=0.01, momentum=0.9), data, 32, 1, 0, None,
                         EngineOptions(graph_steps=5, force_allreduce=True, comm="xgmi", dist_mode=2, plan_world=8))
print("ranges", e.ranges, "xch", e.xch, "comm", e.comm_kind, flush=True)
e.refresh()
e.run_steps(3)
e.synchronize()
print("last_xar", e.eng.last_xar, "fused", e.eng.last_fused_reduce, "fc_role", e.eng.last_fc_role, flush=True)
dist.destroy_process_group()
