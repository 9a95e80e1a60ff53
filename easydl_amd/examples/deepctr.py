"""DeepFM CTR training with row-sparse embedding tables on parameter servers.

The workload of the reference's example job (``elastic-deepctr-job``,
docs/design/elastic-training-operator.md:35-44): PS + workers + evaluator, one
entry point per role (``EDL_ROLE`` set by the local ElasticOperator).  Dense
weights are sharded by bytes over the PS, embedding rows are striped
``id % num_ps`` and updated lazily (Adagrad by default, as CTR jobs do).

Env knobs: EDL_NUM_PS (2), EDL_PS_MODE (async|sync), EDL_BATCH (512),
EDL_SHARD (8192 samples), EDL_EPOCHS (1), EDL_SAMPLES (200000), EDL_VOCAB (10000),
EDL_SPARSE_OPT (adagrad|adam|sgd), EDL_DEVICE (cpu|cuda: PS shards and worker
compute on the rank's GPU).
"""
import json
import os

import torch

from easydl_amd.models.deepctr import DeepFM, SyntheticCTR, auc
from easydl_amd.trainer.context import TrainerContext
from easydl_amd.trainer.ps_trainer import PSWorker, run_evaluator, run_ps


def main():
    torch.set_num_threads(max(1, int(os.environ.get("OMP_NUM_THREADS", 1))))
    ctx = TrainerContext.from_env()
    num_ps = int(os.environ.get("EDL_NUM_PS", 2))
    mode = os.environ.get("EDL_PS_MODE", "async")
    vocab = int(os.environ.get("EDL_VOCAB", 10000))
    dev = os.environ.get("EDL_DEVICE", "cpu")
    if dev == "cuda":
        dev = "cuda:0"  # the operator pins one GPU per role through HIP_VISIBLE_DEVICES
    data = SyntheticCTR(int(os.environ.get("EDL_SAMPLES", 200000)), vocab=vocab)
    model_fn = lambda d: DeepFM(vocab=vocab, device=d)  # noqa: E731
    if ctx.role == "ps":
        run_ps(model_fn, num_ps, ctx, optimizer="adam", lr=1e-3, mode=mode, device=dev,
               sparse_optimizer=os.environ.get("EDL_SPARSE_OPT", "adagrad"), sparse_lr=0.05)
    elif ctx.role == "evaluator":
        run_evaluator(model_fn, num_ps, lambda m: {"auc": auc(m, data, device=dev)}, ctx, interval_s=0.5,
                      device=dev)
    else:
        w = PSWorker(model_fn, num_ps, ctx, device=dev)
        w.fit(lambda m, b: m(*b), data, batch_size=int(os.environ.get("EDL_BATCH", 512)),
              shard_size=int(os.environ.get("EDL_SHARD", 8192)), epochs=int(os.environ.get("EDL_EPOCHS", 1)))
        print(json.dumps({"worker": ctx.index, "steps": w.steps}), flush=True)


if __name__ == "__main__":
    main()
