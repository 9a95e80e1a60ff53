"""Single-GPU sizing run of ONE tensor-parallel shard at full depth (BASELINE.json
config 5: Llama-3 70B, TP=8).

Builds TP rank ``--rank`` of ``--tp`` of the full 80-layer model on this GPU against a
*loopback* TP group (every collective is the identity: all-reduce returns its input,
all-gather replicates it, reduce-scatter takes this rank's slice) and runs real training
steps -- forward, backward, grad-norm clip and the fused AdamW update of every parameter
of the shard, fp32 master weights and moments -- at the batch shape ``bench.py --model
llama3-70b --tp 8`` uses.  What it measures per rank, without the 7 other GPUs:

* peak HBM (allocated and reserved) with and without activation recompute;
* compute ms/step and the projected tokens/s/GPU (TP collectives excluded: their bytes
  per step are reported so the link time can be added from the engine's measurements);
* the in-memory snapshot mode (full / lean / off, ``ckpt/manager.py``) this box's host
  DRAM allows when 8 such ranks share it.

Usage: ``python -m easydl_amd.trainer.tp_dryrun --model llama3-70b --tp 8 --recompute 1``
(one JSON line; ``--out`` also writes it to a file).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
import types

import torch


class LoopbackComm:
    """A TP communicator of ``size`` ranks whose collectives are identities."""

    def __init__(self, size: int, rank: int, device):
        self.world_size, self.rank, self.epoch = size, rank, 0
        self.device = torch.device(device)
        self.backend = "loopback"
        self.aborted = False
        self.bytes = 0          # bytes a real group would have moved through each rank

    def _count(self, t):
        self.bytes += t.numel() * t.element_size()

    def all_reduce(self, t, op=None):
        self._count(t)
        return t

    def all_reduce_async(self, t, op=None):
        self._count(t)
        return types.SimpleNamespace(wait=lambda *a, **k: True, is_completed=lambda: True)

    def wait_work(self, work):
        return None

    def all_gather_into(self, out, inp):
        self._count(out)
        out.view(self.world_size, -1).copy_(inp.reshape(1, -1).expand(self.world_size, -1))
        return out

    def reduce_scatter_into(self, out, inp, op=None):
        self._count(inp)
        out.copy_(inp.reshape(self.world_size, -1)[self.rank].view_as(out))
        return out

    def healthy(self):
        return True


def run(model: str, tp: int, rank: int, seq: int, mbs: int, accum: int, steps: int, warmup: int, recompute: bool,
        sp: bool = False, device: str = "cuda") -> dict:
    from easydl_amd.ckpt.manager import CheckpointManager, shard_layout
    from easydl_amd.models.llama import get_config
    from easydl_amd.optim import FlatAdamW
    from easydl_amd.parallel.flat import FlatBuffers, FlatParams
    from easydl_amd.parallel.tp import LlamaTP, TPGroup

    cuda = device == "cuda"
    dev = torch.device("cuda", 0) if cuda else torch.device("cpu")
    if cuda:
        torch.cuda.set_device(dev)
        torch.cuda.reset_peak_memory_stats(dev)
    sync = (lambda: torch.cuda.synchronize(dev)) if cuda else (lambda: None)  # noqa: E731
    cfg = get_config(model, recompute=recompute)
    comm = LoopbackComm(tp, rank, dev)
    g = TPGroup(comm, sequence_parallel=sp)
    torch.manual_seed(1009 * rank)
    t0 = time.perf_counter()
    m = LlamaTP(cfg, g, device=dev, dtype=torch.bfloat16 if cuda else torch.float32)
    flat = FlatParams(m, weight_decay=0.1)
    bufs = FlatBuffers(m)
    opt = FlatAdamW(flat, lr=3e-4, betas=(0.9, 0.95), weight_decay=0.1, max_grad_norm=1.0)
    w = []
    for grp in flat.groups:
        rep = {bool(getattr(sl.param, "_tp_replicated", False)) for sl in grp.slots}
        w.append(1.0 / tp if rep.pop() else 1.0)
    opt.norm_weights = w
    opt.norm_reduce = lambda t: comm.all_reduce(t)
    sync()
    build_s = time.perf_counter() - t0
    state_gb = (torch.cuda.memory_allocated(dev) if cuda else
                sum(t.numel() * t.element_size() for t in list(m.parameters()) + [grp.grad for grp in flat.groups]
                    + list(opt.state_tensors().values()))) / 2**30
    ids = [torch.randint(0, cfg.vocab_size, (mbs, seq), device=dev) for _ in range(accum)]

    def step():
        flat.zero_grad()
        for x in ids:
            loss = m(x, x) * (1.0 / accum)
            loss.backward()
        flat.finalize_untouched()
        if hasattr(m, "sync_sp_grads"):
            m.sync_sp_grads(flat)
        opt.step()
        return loss

    for _ in range(warmup):
        step()
    sync()
    comm.bytes = 0
    t1 = time.perf_counter()
    for _ in range(steps):
        loss = step()
    sync()
    dt = (time.perf_counter() - t1) / steps
    tokens = mbs * seq * accum                       # per model replica (= per TP group) per step
    fpt = cfg.flops_per_token(seq)
    # the in-memory snapshot this shard would take, and the mode this box's host DRAM allows
    # when 8 ranks share it (LOCAL_WORLD_SIZE = 8: a full TP=8 node)
    tr = types.SimpleNamespace(flat=flat, opt=opt, bufs=bufs, comm=types.SimpleNamespace(world_size=1, rank=0,
                                                                                        epoch=0),
                               step=0, model=m)
    state = CheckpointManager.state_of(tr)
    full = shard_layout(state, 0, 1)[1] + 8
    moments = set(opt.moment_names()) if hasattr(opt, "moment_names") else set()
    lean = shard_layout([(n, t) for n, t in state if n not in moments], 0, 1)[1] + 8
    os.environ["LOCAL_WORLD_SIZE"] = str(tp)
    ck = CheckpointManager("tpdry", interval=1)
    mode = ck._decide_mode(tr, tr.comm, (1, 0, f"-t{rank}of{tp}"), full, lean)
    budget = ck.stats.get("host_budget_gb")
    ck.close()
    return {
        "metric": f"{model} TP={tp} single-shard dry run (TP collectives = identity)",
        "model": model, "tp": tp, "rank": rank, "seq_len": seq, "micro_batch": mbs, "grad_accum": accum,
        "recompute": recompute, "sequence_parallel": sp, "layers": cfg.n_layers,
        "params_per_rank": flat.num_params(), "state_gb": round(state_gb, 2),
        "peak_alloc_gb": round(torch.cuda.max_memory_allocated(dev) / 2**30, 2) if cuda else None,
        "peak_reserved_gb": round(torch.cuda.max_memory_reserved(dev) / 2**30, 2) if cuda else None,
        "hbm_gb": round(torch.cuda.get_device_properties(dev).total_memory / 2**30, 1) if cuda else None,
        "build_s": round(build_s, 2), "ms_per_step": round(dt * 1e3, 1), "steps": steps, "warmup": warmup,
        "tokens_per_step_per_replica": tokens,
        "projected_tokens_per_s_per_gpu": round(tokens / dt / tp, 1),
        "projected_tflops_per_gpu": round(tokens / dt * fpt / tp / 1e12, 1),
        "tp_collective_bytes_per_step_per_rank": comm.bytes // max(1, steps),
        "loss": round(float(loss.detach()) * accum, 4),
        "snapshot": {"full_gb": round(full / 2**30, 2), "lean_gb": round(lean / 2**30, 2),
                     "full_bytes": int(full), "lean_bytes": int(lean),
                     "host_budget_gb_per_rank": budget, "ranks_per_node": tp, "mode": mode,
                     "mem_available_gb": round(_mem_available() / 2**30, 1)},
    }


def _mem_available() -> int:
    with open("/proc/meminfo") as f:
        for ln in f:
            if ln.startswith("MemAvailable:"):
                return int(ln.split()[1]) * 1024
    return 0


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-70b")
    ap.add_argument("--tp", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--seq", type=int, default=8192)
    ap.add_argument("--mbs", type=int, default=1)
    ap.add_argument("--accum", type=int, default=4)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--recompute", type=int, default=1)
    ap.add_argument("--sp", type=int, default=0)
    ap.add_argument("--out", default=None)
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"])
    a = ap.parse_args(argv)
    try:
        res = run(a.model, a.tp, a.rank, a.seq, a.mbs, a.accum, a.steps, a.warmup, bool(a.recompute), bool(a.sp),
                  a.device)
    except torch.OutOfMemoryError as e:   # the answer for this configuration: it does not fit
        res = {"model": a.model, "tp": a.tp, "seq_len": a.seq, "micro_batch": a.mbs, "grad_accum": a.accum,
               "recompute": bool(a.recompute), "oom": True,
               "peak_alloc_gb": round(torch.cuda.max_memory_allocated() / 2**30, 2),
               "hbm_gb": round(torch.cuda.get_device_properties(0).total_memory / 2**30, 1),
               "error": str(e).splitlines()[0][:300]}
    line = json.dumps(res)
    print(line, flush=True)
    if a.out:
        with open(a.out, "a") as f:
            f.write(line + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
