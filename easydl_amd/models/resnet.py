"""ResNet-50 (BASELINE.json config 2: "ResNet-50 bf16 elastic DDP, scale 1->8").

Written here (torchvision is not installed).  bf16 weights in channels-last
memory format so MIOpen picks its NHWC implicit-GEMM (MFMA) convolutions.
Every BatchNorm (fp32 weight and statistics) runs with its ReLU and, at the end
of a bottleneck, the residual add fused in (:func:`easydl_amd.ops.batchnorm.bn_act`,
HIP kernels on the GPU).  Convolutions deliver their weight gradients straight into
the flat gradient buffer; the 1x1 ones run as hipBLASLt GEMMs over the channels-last
pixel matrix (:func:`easydl_amd.ops.conv.conv2d`).  Synthetic ImageNet-shaped data (:class:`SyntheticImages`)
since no dataset can be downloaded.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from easydl_amd.ops import fused
from easydl_amd.ops.batchnorm import bn_act
from easydl_amd.ops.conv import conv2d


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin, width, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, width, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = nn.Conv2d(width, width, 3, stride, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = nn.Conv2d(width, width * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(width * 4)
        nn.init.zeros_(self.bn3.weight)  # zero-init residual branch
        self.downsample = downsample

    def forward(self, x):
        if self.downsample is None:
            idt = x
        else:
            conv, bn = self.downsample
            idt = bn_act(conv2d(x, conv), bn, relu=False)
        y = bn_act(conv2d(x, self.conv1), self.bn1)
        y = bn_act(conv2d(y, self.conv2), self.bn2)
        return bn_act(conv2d(y, self.conv3), self.bn3, residual=idt)


class ResNet(nn.Module):
    def __init__(self, layers=(3, 4, 6, 3), num_classes=1000, width=64):
        super().__init__()
        self.conv1 = nn.Conv2d(3, width, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(width)
        cin = width
        stages = []
        for i, n in enumerate(layers):
            w = width * 2 ** i
            blocks = []
            for j in range(n):
                stride = 2 if (j == 0 and i > 0) else 1
                ds = None
                if j == 0:
                    ds = nn.Sequential(nn.Conv2d(cin, w * 4, 1, stride, bias=False), nn.BatchNorm2d(w * 4))
                blocks.append(Bottleneck(cin, w, stride, ds))
                cin = w * 4
            stages.append(nn.Sequential(*blocks))
        self.stages = nn.Sequential(*stages)
        self.fc = nn.Linear(cin, num_classes)

    def forward(self, x, y=None):
        x = bn_act(conv2d(x, self.conv1), self.bn1)
        x = F.max_pool2d(x, 3, 2, 1)
        x = self.stages(x)
        x = torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)
        logits = fused.linear(x, self.fc.weight, self.fc.bias)
        if y is None:
            return logits
        return F.cross_entropy(logits.float(), y)


def resnet50(device=None, dtype=torch.bfloat16, num_classes=1000) -> ResNet:
    if device is not None and torch.device(device).type == "cuda":
        from easydl_amd.ops import conv_tuning
        conv_tuning.install()   # MIOpen's solver search for these shapes, done once on gfx950
    m = ResNet(num_classes=num_classes)
    m = m.to(device=device, dtype=dtype)
    if device is not None and torch.device(device).type == "cuda":
        m = m.to(memory_format=torch.channels_last)
    for mod in m.modules():  # fp32 weight, bias and batch statistics
        if isinstance(mod, nn.BatchNorm2d):
            mod.float()
    return m


class SyntheticImages:
    def __init__(self, n=1 << 20, size=224, classes=1000, channels_last=True):
        self.n, self.size, self.classes, self.cl = n, size, classes, channels_last

    def __len__(self):
        return self.n

    def batch(self, idx, device="cpu", dtype=torch.bfloat16):
        idx = list(idx)
        g = torch.Generator(device=device).manual_seed(int(idx[0]) if idx else 0)
        x = torch.randn(len(idx), 3, self.size, self.size, device=device, generator=g).to(dtype)
        if self.cl and torch.device(device).type == "cuda":
            x = x.to(memory_format=torch.channels_last)
        y = torch.tensor([(i * 7919) % self.classes for i in idx], device=device)
        return x, y
