"""BERT-large MLM on asynchronous parameter servers (BASELINE.json config 4:
"BERT-large async PS mode, 2 PS + 6 workers, Brain auto CU/HBM plan").

Submitted WITHOUT a JobResource (examples/bert_ps.yaml): the trainer master
extracts the model's features (335 M params -> 4 GB of fp32 state + Adam
moments, 1.3 GB of gradients per push), the Brain plans PS count / workers /
per-PS CU share and HBM cap (easydl_amd/brain/planner.py), the operator
realises the CU share as a CU-masked stream and the cap as an allocator limit.
PS shards live in HBM; with ``EDL_PS_TRANSPORT=ipc`` (default on GPUs) pulls
and pushes move through IPC-mapped HBM (easydl_amd/ps/ipc.py), TCP carries only
control messages.  Workers train bf16 replicas; the PS applies fp32 AdamW.

Env: EDL_NUM_PS (from the plan; default 2), EDL_MODEL (bert-large | bert-tiny),
EDL_SEQ (512), EDL_BATCH (per worker step, 8), EDL_SAMPLES, EDL_SHARD.
"""
import json
import os
import time

import torch

from easydl_amd.models.bert import BERT_LARGE, BERT_TINY, BertMLM, SyntheticMLM
from easydl_amd.trainer.context import TrainerContext
from easydl_amd.trainer.ps_trainer import PSWorker, run_evaluator, run_ps


def main():
    torch.set_num_threads(max(1, int(os.environ.get("OMP_NUM_THREADS", 1))))
    ctx = TrainerContext.from_env()
    num_ps = int(os.environ.get("EDL_NUM_PS", 2))
    cfg = BERT_TINY if "tiny" in os.environ.get("EDL_MODEL", "bert-large") else BERT_LARGE
    seq = int(os.environ.get("EDL_SEQ", 512 if cfg is BERT_LARGE else 64))
    cuda = torch.cuda.is_available() and os.environ.get("EDL_GPU") is not None
    dev = "cuda" if cuda else "cpu"
    if cuda:
        os.environ.setdefault("EDL_PS_TRANSPORT", "ipc")
    data = SyntheticMLM(cfg.vocab_size, seq, n=int(os.environ.get("EDL_SAMPLES", 1 << 16)))
    wdtype = torch.bfloat16 if cuda else torch.float32
    if ctx.role == "ps":
        # the PS keeps fp32 master weights + Adam moments of its shard
        run_ps(lambda d: BertMLM(cfg, device=d, dtype=torch.float32), num_ps, ctx, optimizer="adam", lr=1e-4,
               mode="async", device=dev)
    elif ctx.role == "evaluator":
        batch = data.batch(range(len(data) - 8, len(data)), dev)

        def score(m):
            with torch.no_grad():
                return {"mlm_loss": float(m(*batch))}
        run_evaluator(lambda d: BertMLM(cfg, device=d, dtype=wdtype), num_ps, score, ctx, interval_s=2.0,
                      device=dev)
    else:
        # async PS: pushes pipelined under the next step (bounded staleness, PSWorker)
        w = PSWorker(lambda d: BertMLM(cfg, device=d, dtype=wdtype), num_ps, ctx, device=dev,
                     pipeline=os.environ.get("EDL_PS_PIPELINE", "1") == "1")
        bs = int(os.environ.get("EDL_BATCH", 8))
        losses = {}

        def on_step(wk, loss):   # first loss now (one sync), the last one kept as a tensor
            if "first" not in losses:
                losses["first"] = float(loss.detach())
            losses["last"] = loss.detach()

        t0 = time.perf_counter()
        w.fit(lambda m, b: m(*b), data, batch_size=bs, shard_size=int(os.environ.get("EDL_SHARD", 64)),
              epochs=1, on_step=on_step)
        dt = time.perf_counter() - t0
        res = {"worker": ctx.index, "steps": w.steps, "samples_per_s": round(w.steps * bs / dt, 2),
               "transport": w.client.transport, "pipeline": w.pipeline, "versions": list(w.client.versions),
               "first_loss": losses.get("first"),
               "last_loss": float(losses["last"]) if "last" in losses else None}
        w.events.emit("worker_done", **res)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
