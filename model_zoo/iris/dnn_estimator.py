"""Iris DNN classifier with parameter servers -- the reference example's entry point.

The reference's example ElasticJob (docs/design/elastic-training-operator.md:31-45)
sets ``command: "python -m model_zoo.iris.dnn_estimator"`` for its PS, worker and
evaluator roles.  This module is that command for the local operator: the
operator sets ``EDL_ROLE`` and the same process image serves a PS shard, trains
or evaluates.  The data are the 150 Iris samples that scikit-learn ships inside
its package (no download).  They are standardised, and samples are drawn with
replacement so a job can run any number of steps (``EDL_SAMPLES``, default 30000).
A fixed-seed synthetic 4-feature / 3-class set stands in when scikit-learn is
absent.  Model: MLP 4 -> 64 -> 64 -> 3 (``easydl_amd.models.mlp.MLP``).
Env knobs: EDL_NUM_PS (1), EDL_PS_MODE (async|sync), EDL_BATCH (32),
EDL_SHARD (512 samples), EDL_EPOCHS (1), EDL_SAMPLES (30000).
"""
from __future__ import annotations

import json
import os

import torch

from easydl_amd.models.mlp import MLP
from easydl_amd.trainer.context import TrainerContext
from easydl_amd.trainer.ps_trainer import PSWorker, run_evaluator, run_ps


def _iris_arrays() -> tuple[torch.Tensor, torch.Tensor]:
    try:
        from sklearn.datasets import load_iris
        d = load_iris()
        x = torch.tensor(d.data, dtype=torch.float32)
        y = torch.tensor(d.target, dtype=torch.long)
    except Exception:   # scikit-learn missing: a separable stand-in of the same shape
        g = torch.Generator().manual_seed(0)
        y = torch.arange(150) % 3
        x = torch.randn(3, 4, generator=g)[y] * 2 + 0.5 * torch.randn(150, 4, generator=g)
    x = (x - x.mean(0)) / x.std(0)
    return x, y


class IrisData:
    """``n`` draws (with replacement, fixed permutation) from the 150 Iris samples."""

    def __init__(self, n: int = 30000, seed: int = 0):
        self.x, self.y = _iris_arrays()
        g = torch.Generator().manual_seed(seed)
        self.order = torch.randint(0, len(self.y), (n,), generator=g)
        self.n = n

    def __len__(self):
        return self.n

    def batch(self, idx, device="cpu"):
        sel = self.order[torch.as_tensor(list(idx), dtype=torch.long)]
        return self.x[sel].to(device), self.y[sel].to(device)

    def all(self, device="cpu"):
        return self.x.to(device), self.y.to(device)


def make_model(device=None) -> MLP:
    return MLP(inp=4, hidden=(64, 64), classes=3, device=device)


def accuracy(model, data: IrisData) -> float:
    with torch.no_grad():
        x, y = data.all()
        return (model(x).argmax(-1) == y).float().mean().item()


def main():
    torch.set_num_threads(max(1, int(os.environ.get("OMP_NUM_THREADS", 1))))
    ctx = TrainerContext.from_env()
    num_ps = int(os.environ.get("EDL_NUM_PS", 1))
    mode = os.environ.get("EDL_PS_MODE", "async")
    data = IrisData(int(os.environ.get("EDL_SAMPLES", 30000)))
    if ctx.role == "ps":
        run_ps(make_model, num_ps, ctx, optimizer="adam", lr=1e-2, mode=mode)
    elif ctx.role == "evaluator":
        run_evaluator(make_model, num_ps, lambda m: {"acc": accuracy(m, data)}, ctx, interval_s=0.5)
    else:
        w = PSWorker(make_model, num_ps, ctx)
        w.fit(lambda m, b: m(*b), data, batch_size=int(os.environ.get("EDL_BATCH", 32)),
              shard_size=int(os.environ.get("EDL_SHARD", 512)), epochs=int(os.environ.get("EDL_EPOCHS", 1)))
        print(json.dumps({"worker": ctx.index, "steps": w.steps, "acc": round(accuracy(w.model.eval(), data), 4)}),
              flush=True)


if __name__ == "__main__":
    main()
