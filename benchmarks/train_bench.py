#!/usr/bin/env python
"""Throughput benchmarks of the other BASELINE.json configs through ElasticTrainer.

    python benchmarks/train_bench.py --model resnet50 --batch 256      # config 2: images/s
    python benchmarks/train_bench.py --model bert-large --batch 32     # config 4 model, DDP: samples/s
    python benchmarks/train_bench.py --model llama3-8b --batch 4       # config 3 (== bench.py)
Runs under torchrun for N GPUs exactly like bench.py (weak scaling; synthetic
data, random init).  Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=256, help="per-GPU samples per step")
    ap.add_argument("--micro", type=int, default=0, help="micro-batch (default = batch)")
    ap.add_argument("--seq", type=int, default=512)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    a = ap.parse_args()
    t_start = time.perf_counter()
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    dev = torch.device("cuda", local) if torch.cuda.is_available() else torch.device("cpu")
    os.environ.setdefault("EDL_JOB", f"bench-{a.model}")
    os.environ.setdefault("EDL_RUN_DIR", f"gpurun_out/bench_{a.model}")
    from easydl_amd.trainer.elastic import ElasticTrainer
    micro = a.micro or a.batch
    if a.model == "resnet50":
        from easydl_amd.models.resnet import SyntheticImages, resnet50
        model_fn = lambda d: resnet50(d)  # noqa: E731
        data = SyntheticImages()
        unit, per_sample, opt = "images/s", 1, dict(optimizer="sgd", lr=0.1, momentum=0.9, weight_decay=5e-5,
                                                     max_grad_norm=0.0)
        loss_fn = lambda m, b: m(*b)  # noqa: E731
    elif a.model.startswith("bert"):
        from easydl_amd.models.bert import BERT_LARGE, BertMLM, SyntheticMLM
        model_fn = lambda d: BertMLM(BERT_LARGE, device=d)  # noqa: E731
        data = SyntheticMLM(BERT_LARGE.vocab_size, a.seq)
        unit, per_sample, opt = "samples/s", 1, dict(lr=1e-4)
        loss_fn = lambda m, b: m(*b)  # noqa: E731
    else:
        from easydl_amd.models.llama import Llama, get_config
        from easydl_amd.trainer.data import SyntheticTokens
        cfg = get_config(a.model)
        model_fn = lambda d: Llama(cfg, device=d)  # noqa: E731
        data = SyntheticTokens(cfg.vocab_size, a.seq)
        unit, per_sample, opt = "tokens/s", a.seq, dict(lr=3e-4)
        loss_fn = lambda m, b: m(*b)  # noqa: E731
    tr = ElasticTrainer(model_fn, global_batch=world * a.batch, micro_batch=micro, device=dev, **opt)
    marks = {}

    def on_step(t, loss):
        if t.step in (a.warmup, a.warmup + a.steps):
            if dev.type == "cuda":
                torch.cuda.synchronize(dev)
            t.comm.barrier()
            marks[t.step] = time.perf_counter()

    tr.fit(loss_fn, data, num_steps=a.warmup + a.steps, on_step=on_step)
    el = marks[a.warmup + a.steps] - marks[a.warmup]
    if tr.comm.world_size > 1:
        import torch.distributed as dist
        el = float(tr.comm.ctrl_all_reduce([el], op=dist.ReduceOp.MAX)[0])
    val = tr.comm.world_size * a.batch * per_sample * a.steps / el
    if tr.comm.rank == 0:
        print(json.dumps({"metric": f"{unit} {a.model} elastic DDP", "value": round(val, 2), "unit": unit,
                          "n_gpus": tr.comm.world_size, "steps": a.steps, "warmup": a.warmup,
                          "ms_per_step": round(el / a.steps * 1e3, 2), "per_gpu_batch": a.batch, "micro": micro,
                          "seq": a.seq if a.model != "resnet50" else None, "dtype": "bf16",
                          "loss": round(float(tr.last_loss), 4),
                          "setup_and_warmup_s": round(marks[a.warmup] - t_start, 2),
                          "peak_mem_gb": round(torch.cuda.max_memory_allocated(dev) / 2**30, 1)
                          if dev.type == "cuda" else 0}), flush=True)
    tr.close()


if __name__ == "__main__":
    main()
