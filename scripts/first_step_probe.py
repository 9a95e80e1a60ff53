"""Where does a fresh process's first Llama-3-8B step go (host enqueue vs GPU), and how much of it
can be warmed up beforehand?  Runs one process per mode (call once per mode):

  cold   build the full model, time the first two steps
  warm   first build a 1-layer model of the same width and run one step (every GEMM shape, kernel and
         hipBLASLt solution the full model uses, plus allocator growth), free it, then as `cold`

Prints one JSON line per mode.  (A no-survivor replacement pays the cold first step: 1.2 s vs 0.4 s.)"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from easydl_amd.models.llama import Llama, get_config  # noqa: E402
from easydl_amd.trainer.data import SyntheticTokens  # noqa: E402
from easydl_amd.trainer.elastic import ElasticTrainer  # noqa: E402


def trainer(cfg):
    return ElasticTrainer(lambda d: Llama(cfg, device=d), global_batch=1, micro_batch=1,
                          device=torch.device("cuda", 0))


def step_times(tr, data, n):
    """Per step: host time to get through the step (enqueue) and time until the GPU is done."""
    out, t = [], [None]

    def on_step(trainer, loss):
        th = time.perf_counter()
        torch.cuda.synchronize()
        out.append({"host_s": round(th - t[0], 3), "total_s": round(time.perf_counter() - t[0], 3)})
        t[0] = time.perf_counter()

    torch.cuda.synchronize()
    t[0] = time.perf_counter()
    tr.fit(lambda m, b: m(*b), data, num_steps=tr.step + n, on_step=on_step)
    return out


def main():
    mode = sys.argv[1]
    cfg = get_config("llama3-8b")
    data = SyntheticTokens(cfg.vocab_size, 8192, num_samples=64)
    res = {"mode": mode}
    if mode == "warm":
        t0 = time.perf_counter()
        small = trainer(get_config("llama3-8b", n_layers=1))
        res["warm_steps"] = step_times(small, data, 1)
        del small
        torch.cuda.synchronize()
        res["warmup_s"] = round(time.perf_counter() - t0, 3)
    t0 = time.perf_counter()
    tr = trainer(cfg)
    res["build_s"] = round(time.perf_counter() - t0, 3)
    res["steps"] = step_times(tr, data, 3)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
