"""Stock PyTorch-ROCm ResNet-18 training step (MIOpen convs, autocast bf16, channels_last)
at the same batch / image size as `bench.py --model resnet18`, as the comparison point for
our HIP module path.  torchvision is not installed, so the network is defined here
(standard ResNet-18: 7x7/2 stem, maxpool, 4 stages x 2 BasicBlocks, avgpool, fc 1000).

    python scripts/resnet_torch_ref.py --steps 30 --warmup 10 [--batch_size 32]
"""
import argparse
import json
import time

import torch
import torch.nn as nn
import torch.nn.functional as F


class Block(nn.Module):
    def __init__(self, cin, cout, stride):
        super().__init__()
        self.c1 = nn.Conv2d(cin, cout, 3, stride, 1, bias=False)
        self.b1 = nn.BatchNorm2d(cout)
        self.c2 = nn.Conv2d(cout, cout, 3, 1, 1, bias=False)
        self.b2 = nn.BatchNorm2d(cout)
        self.down = None
        if stride != 1 or cin != cout:
            self.down = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))

    def forward(self, x):
        y = F.relu(self.b1(self.c1(x)))
        y = self.b2(self.c2(y))
        return F.relu(y + (x if self.down is None else self.down(x)))


class ResNet18(nn.Module):
    def __init__(self):
        super().__init__()
        self.stem = nn.Sequential(nn.Conv2d(3, 64, 7, 2, 3, bias=False), nn.BatchNorm2d(64), nn.ReLU(),
                                  nn.MaxPool2d(3, 2, 1))
        layers, cin = [], 64
        for cout, s in ((64, 1), (128, 2), (256, 2), (512, 2)):
            layers += [Block(cin, cout, s), Block(cout, cout, 1)]
            cin = cout
        self.layers = nn.Sequential(*layers)
        self.fc = nn.Linear(512, 1000)

    def forward(self, x):
        x = self.layers(self.stem(x))
        return self.fc(torch.flatten(F.adaptive_avg_pool2d(x, 1), 1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch_size", type=int, default=32)
    ap.add_argument("--image_size", type=int, default=224)
    ap.add_argument("--no_channels_last", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.backends.cudnn.benchmark = True
    torch.manual_seed(0)
    fmt = torch.contiguous_format if a.no_channels_last else torch.channels_last
    model = ResNet18().to(dev).to(memory_format=fmt)
    opt = torch.optim.SGD(model.parameters(), lr=0.01, momentum=0.9)
    xs = [torch.randn(a.batch_size, 3, a.image_size, a.image_size, device=dev).to(memory_format=fmt)
          for _ in range(4)]
    ys = [torch.randint(0, 1000, (a.batch_size,), device=dev) for _ in range(4)]

    def step(i):
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = F.cross_entropy(model(xs[i % 4]), ys[i % 4])
        loss.backward()
        opt.step()
        return loss

    for i in range(a.warmup):
        step(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        loss = step(i)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(json.dumps({"metric": "images/sec ResNet-18 (stock PyTorch-ROCm, autocast bf16)",
                      "value": round(a.batch_size * a.steps / dt, 1), "ms_per_step": round(dt * 1e3 / a.steps, 4),
                      "batch": a.batch_size, "image_size": a.image_size,
                      "channels_last": not a.no_channels_last, "loss": round(float(loss), 4)}), flush=True)


if __name__ == "__main__":
    main()
