"""MNIST MLP with parameter servers (BASELINE.json config 1).

One entry point for every role; the local ElasticOperator sets ``EDL_ROLE``:
    ps -> serve a shard,  worker -> train,  evaluator -> score periodically.
Env knobs: EDL_NUM_PS (default 1), EDL_PS_MODE (async|sync), EDL_BATCH (64),
EDL_SHARD (1024 samples), EDL_EPOCHS (1), EDL_SAMPLES (20000).
"""
import json
import os

import torch

from easydl_amd.models.mlp import MLP, SyntheticMNIST, accuracy
from easydl_amd.trainer.context import TrainerContext
from easydl_amd.trainer.ps_trainer import PSWorker, run_evaluator, run_ps


def main():
    torch.set_num_threads(max(1, int(os.environ.get("OMP_NUM_THREADS", 1))))
    ctx = TrainerContext.from_env()
    num_ps = int(os.environ.get("EDL_NUM_PS", 1))
    mode = os.environ.get("EDL_PS_MODE", "async")
    data = SyntheticMNIST(int(os.environ.get("EDL_SAMPLES", 20000)))
    model_fn = lambda dev: MLP(device=dev)  # noqa: E731
    if ctx.role == "ps":
        run_ps(model_fn, num_ps, ctx, optimizer="adam", lr=1e-3, mode=mode)
    elif ctx.role == "evaluator":
        run_evaluator(model_fn, num_ps, lambda m: {"acc": accuracy(m, data)}, ctx, interval_s=0.5)
    else:
        w = PSWorker(model_fn, num_ps, ctx)
        w.fit(lambda m, b: m(*b), data, batch_size=int(os.environ.get("EDL_BATCH", 64)),
              shard_size=int(os.environ.get("EDL_SHARD", 1024)), epochs=int(os.environ.get("EDL_EPOCHS", 1)))
        acc = accuracy(w.model.eval(), data) if False else None
        print(json.dumps({"worker": ctx.index, "steps": w.steps}), flush=True)


if __name__ == "__main__":
    main()
