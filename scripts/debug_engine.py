import faulthandler, sys, os
faulthandler.enable()
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from ddp_amd.data import DeviceMNIST, synthetic_mnist
from ddp_amd.engine import EngineOptions, FusedSimpleCNNEngine
from ddp_amd.models import SimpleCNN
from ddp_amd.ops import FusedSGD
def p(*a): print(*a, flush=True, file=sys.stderr)
dev = torch.device("cuda", 0)
torch.manual_seed(0)
model = SimpleCNN().to(dev)
opt = FusedSGD(model, lr=0.01)
imgs, labels = synthetic_mnist(2048)
data = DeviceMNIST(imgs, labels, dev)
p("creating engine")
eng = FusedSimpleCNNEngine(model, opt, data, 32, 1, 0, opts=EngineOptions(graph_steps=int(sys.argv[1]) if len(sys.argv) > 1 else 2))
p("refresh"); eng.refresh(); eng.synchronize()
p("eager steps"); eng.run_steps(0); eng.eng.step(32, 32); eng.synchronize()
p("capture"); eng.eng.capture(eng.opts.graph_steps); p("captured")
eng.eng.replay(); p("replayed"); eng.synchronize(); p("synced", torch.isfinite(eng.fs.params).all().item())
