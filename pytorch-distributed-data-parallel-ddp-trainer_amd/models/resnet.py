"""ResNet-18 (BASELINE.json config 5: synthetic 3x224x224, DDP stress of the bucketed
all-reduce and the MFMA convolutions).

Module tree and ``state_dict`` names follow torchvision's ``resnet18`` (conv1, bn1,
layer1..4 of BasicBlocks with ``downsample.0/1``, fc), so torchvision checkpoints
load; conv weights live as native OHWI tensors (see layers.Conv2d).

* CUDA input: NHWC bf16 pipeline on the HIP kernels of ``ops/resnet_fn.py`` -
  every conv is conv+BN(+residual)+ReLU fused into one autograd Function whose
  convolution carries the BatchNorm batch statistics in its epilogue.
* CPU input: plain fp32 PyTorch (NCHW) - the reference/oracle path.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from .layers import Conv2d, Linear


def _init_conv(conv: Conv2d):
    """torchvision init: kaiming_normal_(fan_out, relu) on the OIHW tensor."""
    w = torch.empty(conv.out_channels, conv.in_channels, conv.kernel_size, conv.kernel_size)
    nn.init.kaiming_normal_(w, mode="fan_out", nonlinearity="relu")
    with torch.no_grad():
        conv.weight.copy_(w.permute(0, 2, 3, 1))


def conv3x3(cin, cout, stride=1):
    c = Conv2d(cin, cout, 3, stride=stride, padding=1, bias=False)
    _init_conv(c)
    return c


def conv1x1(cin, cout, stride=1):
    c = Conv2d(cin, cout, 1, stride=stride, padding=0, bias=False)
    _init_conv(c)
    return c


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, cin, cout, stride=1):
        super().__init__()
        self.conv1 = conv3x3(cin, cout, stride)
        self.bn1 = nn.BatchNorm2d(cout)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = conv3x3(cout, cout)
        self.bn2 = nn.BatchNorm2d(cout)
        self.downsample = None
        if stride != 1 or cin != cout:
            self.downsample = nn.Sequential(conv1x1(cin, cout, stride), nn.BatchNorm2d(cout))

    def forward_nchw(self, x):
        idt = x
        out = self.relu(self.bn1(self.conv1.forward_nchw(x)))
        out = self.bn2(self.conv2.forward_nchw(out))
        if self.downsample is not None:
            idt = self.downsample[1](self.downsample[0].forward_nchw(x))
        return self.relu(out + idt)

    def forward_hip(self, x):
        from ..ops.resnet_fn import attach_stash, conv_bn_act

        # x feeds two branches: the residual one hands its gradient to x's producer, which
        # adds it inside its own backward (no separate gradient-add kernel)
        stash = attach_stash(x) if torch.is_grad_enabled() and x.requires_grad else None
        out = conv_bn_act(x, self.conv1, self.bn1, relu=True, defer=True)  # BN + ReLU in conv2's loads
        if self.downsample is not None:
            idt = conv_bn_act(x, self.downsample[0], self.downsample[1], relu=False, stash=stash)
            return conv_bn_act(out, self.conv2, self.bn2, res=idt, relu=True)
        return conv_bn_act(out, self.conv2, self.bn2, res=x, relu=True, stash=stash)


class ResNet(nn.Module):
    def __init__(self, layers=(2, 2, 2, 2), num_classes=1000):
        super().__init__()
        self.conv1 = Conv2d(3, 64, 7, stride=2, padding=3, bias=False)
        _init_conv(self.conv1)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        cin = 64
        for i, (cout, n) in enumerate(zip((64, 128, 256, 512), layers)):
            blocks = []
            for j in range(n):
                stride = 2 if (j == 0 and i > 0) else 1
                blocks.append(BasicBlock(cin, cout, stride))
                cin = cout
            setattr(self, f"layer{i + 1}", nn.Sequential(*blocks))
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = Linear(512, num_classes)
        bound = 1.0 / math.sqrt(512)
        with torch.no_grad():
            self.fc.weight.uniform_(-bound, bound)
            self.fc.bias.uniform_(-bound, bound)

    def blocks(self):
        for i in range(1, 5):
            yield from getattr(self, f"layer{i}")

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if x.is_cuda:
            return self.forward_hip(x)
        h = self.maxpool(self.relu(self.bn1(self.conv1.forward_nchw(x))))
        for b in self.blocks():
            h = b.forward_nchw(h)
        return self.fc(torch.flatten(self.avgpool(h), 1))

    def forward_hip(self, x: torch.Tensor) -> torch.Tensor:
        """x: NCHW float [B,3,H,W] or already NHWC4 bf16 [B,H,W,4]."""
        from ..ops import resnet_fn as R

        if x.dim() == 4 and x.shape[1] == 3:
            x = R.to_nhwc4(x)
        h = R.conv_bn_act(x, self.conv1, self.bn1, relu=True, defer=True)  # BN + ReLU in the maxpool
        h = R.maxpool3x3s2(h)
        for b in self.blocks():
            h = b.forward_hip(h)
        return R.linear_head(R.global_avgpool(h), self.fc.weight, self.fc.bias)


def resnet18(num_classes: int = 1000) -> ResNet:
    return ResNet((2, 2, 2, 2), num_classes)
