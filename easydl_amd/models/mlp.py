"""MNIST-style MLP (BASELINE.json config 1: "MNIST MLP, 1 PS + 2 workers on CPU/gloo").

No network is available for the real MNIST download, so :class:`SyntheticMNIST`
generates a deterministic 10-class problem of 28x28 "images" (class prototypes
+ pixel noise): learnable, so accuracy is a meaningful end-to-end signal.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


class MLP(nn.Module):
    def __init__(self, inp: int = 784, hidden=(256, 256), classes: int = 10, device=None, dtype=torch.float32):
        super().__init__()
        dims = [inp, *hidden, classes]
        self.layers = nn.ModuleList(nn.Linear(a, b, device=device, dtype=dtype) for a, b in zip(dims[:-1], dims[1:]))

    def forward(self, x, y=None):
        x = x.reshape(x.shape[0], -1)
        for i, l in enumerate(self.layers):
            x = l(x)
            if i < len(self.layers) - 1:
                x = F.relu(x)
        if y is None:
            return x
        return F.cross_entropy(x.float(), y)


class SyntheticMNIST:
    def __init__(self, n: int = 60000, seed: int = 0, noise: float = 0.9):
        g = torch.Generator().manual_seed(seed)
        self.protos = torch.randn(10, 784, generator=g)
        self.n, self.seed, self.noise = n, seed, noise

    def __len__(self):
        return self.n

    def batch(self, idx, device="cpu"):
        idx = torch.as_tensor(list(idx), dtype=torch.long)
        y = (idx * 7919 + self.seed) % 10
        g = torch.Generator().manual_seed(int(self.seed * 1_000_003 + int(idx[0]) if len(idx) else 0))
        x = self.protos[y] + self.noise * torch.randn(len(idx), 784, generator=g)
        return x.view(-1, 1, 28, 28).to(device), y.to(device)


def accuracy(model, data: SyntheticMNIST, n: int = 2000, device="cpu") -> float:
    with torch.no_grad():
        x, y = data.batch(range(data.n - n, data.n), device)
        return (model(x).argmax(-1) == y).float().mean().item()
