#!/usr/bin/env python
"""Headline benchmark: Llama-3-8B elastic-DDP training throughput (tokens/s).

Metric/config come from BASELINE.json (``tokens/sec ... Llama-3-8B elastic
DDP 1->8 GPUs``).  One process per GPU; for N>1 the driver launches this file
with ``torch.distributed.run`` and every rank reads RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_ADDR / MASTER_PORT from the environment.

Each timed step is a COMPLETE training step of the full 32-layer Llama-3-8B
architecture (random init, synthetic tokens): forward, backward with the
bucketed RCCL all-reduce overlapped, global grad-norm clip and the fused
AdamW update of all 8.03e9 parameters (fp32 master + moments).  W untimed
warmup steps, then exactly K steps bracketed by barrier + synchronize; the
elapsed time is the MAX over ranks; rank 0 prints one JSON line.

``--fault-inject`` additionally measures time-to-recover (see
``easydl_amd/trainer/fault_bench.py``) — not part of the default run.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--seq", type=int, default=8192)
    ap.add_argument("--mbs", type=int, default=1, help="sequences per micro-batch per GPU")
    ap.add_argument("--accum", type=int, default=1, help="micro-batches per step")
    ap.add_argument("--bucket-mb", type=float, default=None)
    ap.add_argument("--layers", type=int, default=None, help="override layer count (debug only; invalid for the metric)")
    ap.add_argument("--profile-steps", type=int, default=0)
    ap.add_argument("--out", default=None)
    return ap.parse_args()


def main():
    args = parse()
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if world != args.gpus and rank == 0:
        print(f"[bench] note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    use_cuda = torch.cuda.is_available()
    dev = torch.device("cuda", local) if use_cuda else torch.device("cpu")
    if use_cuda:
        torch.cuda.set_device(dev)

    from easydl_amd.models.llama import Llama, get_config
    from easydl_amd.optim import FlatAdamW
    from easydl_amd.parallel.comm import Communicator, LocalCommunicator
    from easydl_amd.parallel.ddp import ElasticDDP
    from easydl_amd.parallel.flat import FlatParams

    comm = LocalCommunicator(dev)
    if world > 1:
        import torch.distributed as dist
        import datetime
        addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
        port = int(os.environ.get("MASTER_PORT", 29500))
        agent_store = os.environ.get("TORCHELASTIC_USE_AGENT_STORE", "") in ("True", "true", "1")
        store = dist.TCPStore(addr, port, world, is_master=(rank == 0 and not agent_store),
                              timeout=datetime.timedelta(seconds=300))
        comm = Communicator(store, rank, world, epoch=0, device=dev, job="bench")
        comm.warmup()

    overrides = {}
    if args.layers:
        overrides["n_layers"] = args.layers
    cfg = get_config(args.model, **overrides)
    torch.manual_seed(1234)  # identical init on every rank (also re-broadcast below)
    model = Llama(cfg, device=dev, dtype=torch.bfloat16 if use_cuda else torch.float32)
    flat = FlatParams(model, weight_decay=0.1)
    ddp = ElasticDDP(flat, comm, bucket_mb=args.bucket_mb)
    ddp.broadcast_params(0)
    opt = FlatAdamW(flat, lr=3e-4, betas=(0.9, 0.95), weight_decay=0.1, max_grad_norm=1.0)

    S, B = args.seq, args.mbs
    g = torch.Generator(device=dev)
    g.manual_seed(42 + rank)
    batches = [(torch.randint(0, cfg.vocab_size, (B, S), device=dev, generator=g),
                torch.randint(0, cfg.vocab_size, (B, S), device=dev, generator=g)) for _ in range(2)]

    def train_step(i):
        flat.zero_grad()
        for a in range(args.accum):
            ids, labels = batches[(i + a) % 2]
            if a < args.accum - 1:
                with ddp.no_sync():
                    loss = model(ids, labels)
                    loss.backward()
            else:
                loss = model(ids, labels)
                loss.backward()
        ddp.finish()
        opt.step(pre_scale=1.0 / (comm.world_size * args.accum))
        return loss

    def sync():
        if use_cuda:
            torch.cuda.synchronize(dev)
        comm.barrier()

    t_w = time.perf_counter()
    for i in range(args.warmup):
        loss = train_step(i)
    sync()
    warm_s = time.perf_counter() - t_w
    if args.profile_steps:
        for i in range(args.profile_steps):
            train_step(i)
        sync()

    sync()
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss = train_step(i)
    sync()
    el = time.perf_counter() - t0
    el_max = float(comm.ctrl_all_reduce([el], op=__import__("torch.distributed", fromlist=["ReduceOp"]).ReduceOp.MAX)[0]) \
        if world > 1 else el
    loss_v = float(loss)
    tokens = comm.world_size * B * S * args.accum * args.steps
    tps = tokens / el_max
    ms = el_max / args.steps * 1e3
    fpt = cfg.flops_per_token(S)
    tflops_gpu = tps / comm.world_size * fpt / 1e12
    mem_gb = torch.cuda.max_memory_allocated(dev) / 2**30 if use_cuda else 0.0
    res = {
        "metric": "tokens/sec, Llama-3-8B elastic DDP (full train step: fwd+bwd+allreduce+AdamW)",
        "value": round(tps, 2),
        "unit": "tokens/s",
        "n_gpus": comm.world_size,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic (random token ids), random-init weights",
        "config": {
            "model": args.model if not args.layers else f"{args.model}-L{args.layers}",
            "global_batch": comm.world_size * B * args.accum,
            "seq_len": S,
            "parallelism": f"dp{comm.world_size}",
            "micro_batch": B,
            "grad_accum": args.accum,
            "optimizer": "AdamW fp32 master/moments, clip 1.0",
            "bucket_mb": ddp.bucket_mb,
        },
        "tflops_per_gpu": round(tflops_gpu, 1),
        "mfu_vs_2.5PF": round(tflops_gpu / 2500.0, 4),
        "loss": round(loss_v, 4),
        "peak_mem_gb": round(mem_gb, 1),
        "warmup_s": round(warm_s, 2),
        "time_to_recover_s": None,
    }
    if rank == 0:
        line = json.dumps(res)
        print(line, flush=True)
        if args.out:
            with open(args.out, "w") as f:
                f.write(line + "\n")
    comm.shutdown()


if __name__ == "__main__":
    main()
