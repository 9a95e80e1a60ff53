"""Elastic data dispatch for all-reduce training.

Every step consumes exactly ``global_batch`` samples from a global,
seeded permutation, whatever the world size; rank r of W takes positions
``r, r+W, ...`` of the step's window and splits them into micro-batches.  A
resize therefore neither drops nor duplicates a sample (SURVEY.md §7.3 item 9,
B11): the only cursor is the committed global step, which every rank agrees
on through the step-commit protocol.  Gradient contributions are weighted by
``len(micro_batch) / global_batch`` so the summed all-reduce equals the
global-batch mean exactly, including uneven splits.
"""
from __future__ import annotations

import math

import torch


class ElasticBatchPlan:
    def __init__(self, num_samples: int, global_batch: int, micro_batch: int, seed: int = 0, shuffle: bool = True):
        self.n = num_samples
        self.global_batch = global_batch
        self.micro_batch = micro_batch
        self.seed = seed
        self.shuffle = shuffle
        self._perm_epoch = -1
        self._perm = None

    def steps_per_epoch(self) -> int:
        return max(1, self.n // self.global_batch)

    _MATERIALIZE_MAX = 1 << 24

    def _perm_for(self, epoch: int):
        if self._perm_epoch != epoch:
            if not self.shuffle:
                self._perm = None
            elif self.n <= self._MATERIALIZE_MAX:
                g = torch.Generator().manual_seed(self.seed * 1000003 + epoch)
                self._perm = torch.randperm(self.n, generator=g)
            else:
                # huge index spaces: seeded affine bijection i -> (a*i + b) mod n, no memory
                import random
                r = random.Random(self.seed * 1000003 + epoch)
                while True:
                    a = r.randrange(1, self.n)
                    if math.gcd(a, self.n) == 1:
                        break
                self._perm = (a, r.randrange(0, self.n))
            self._perm_epoch = epoch
        return self._perm

    def _take(self, perm, lo: int, hi: int) -> torch.Tensor:
        if perm is None:
            return torch.arange(lo, hi)
        if isinstance(perm, tuple):
            a, b = perm
            return torch.tensor([(a * i + b) % self.n for i in range(lo, hi)], dtype=torch.long)
        return perm[lo:hi]

    def indices(self, step: int, rank: int, world: int) -> list[list[int]]:
        """Micro-batches (lists of sample indices) of ``rank`` at global ``step``."""
        spe = self.steps_per_epoch()
        epoch, k = divmod(step, spe)
        perm = self._perm_for(epoch)
        window = self._take(perm, k * self.global_batch, (k + 1) * self.global_batch)
        mine = window[rank::world].tolist()
        return [mine[i:i + self.micro_batch] for i in range(0, len(mine), self.micro_batch)]


class SyntheticTokens:
    """Deterministic synthetic LM samples: sample i -> (ids, labels) of length ``seq``."""

    def __init__(self, vocab: int, seq: int, num_samples: int = 1 << 30):
        self.vocab, self.seq, self.n = vocab, seq, num_samples

    def __len__(self):
        return self.n

    def batch(self, idx: list[int], device) -> tuple[torch.Tensor, torch.Tensor]:
        g = torch.Generator(device=device)
        out = torch.empty(len(idx), self.seq + 1, dtype=torch.long, device=device)
        for j, i in enumerate(idx):
            g.manual_seed(1_000_003 + int(i))
            out[j] = torch.randint(0, self.vocab, (self.seq + 1,), device=device, generator=g)
        return out[:, :-1], out[:, 1:]


class DatasetSource:
    """Wraps a map-style dataset + collate into the ``batch(idx, device)`` interface."""

    def __init__(self, dataset, collate=None):
        self.dataset = dataset
        self.collate = collate or torch.utils.data.default_collate

    def __len__(self):
        return len(self.dataset)

    def batch(self, idx, device):
        b = self.collate([self.dataset[i] for i in idx])
        return _to(b, device)


def _to(b, device):
    if isinstance(b, torch.Tensor):
        return b.to(device, non_blocking=True)
    if isinstance(b, (list, tuple)):
        return type(b)(_to(x, device) for x in b)
    if isinstance(b, dict):
        return {k: _to(v, device) for k, v in b.items()}
    return b
