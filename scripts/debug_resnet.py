"""GPU diagnostic: per-parameter gradient error of the HIP ResNet-18 vs fp32 CPU, next
to the error of a bf16 CPU run vs the same fp32 CPU run (the precision floor)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F

from ddp_amd.models import resnet18
from ddp_amd.ops import CrossEntropyLoss


def relerr(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


def main(bs=4, hw=64):
    torch.manual_seed(0)
    dev = torch.device("cuda", 0)
    cpu = resnet18(num_classes=10)
    cpu16 = resnet18(num_classes=10)
    cpu16.load_state_dict(cpu.state_dict())
    gpu = resnet18(num_classes=10).to(dev)
    gpu.load_state_dict(cpu.state_dict())
    x = torch.randn(bs, 3, hw, hw)
    y = torch.randint(0, 10, (bs,))
    lc = F.cross_entropy(cpu(x), y)
    lc.backward()
    cpu16 = cpu16.to(torch.bfloat16)
    l16 = F.cross_entropy(cpu16(x.to(torch.bfloat16)).float(), y)
    l16.backward()
    lg = CrossEntropyLoss()(gpu(x.to(dev)), y.to(dev))
    lg.backward()
    print(f"bs={bs} hw={hw} loss cpu={lc.item():.5f} cpu_bf16={l16.item():.5f} hip={lg.item():.5f}")
    for (n, pc), (_, p16), (_, pg) in zip(cpu.named_parameters(), cpu16.named_parameters(),
                                          gpu.named_parameters()):
        print(f"{n:32s} hip {relerr(pg.grad, pc.grad):.4f}   cpu_bf16 {relerr(p16.grad, pc.grad):.4f}")


if __name__ == "__main__":
    main(4, 64)
    main(16, 64)
