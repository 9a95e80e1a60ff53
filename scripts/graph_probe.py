"""How launch-bound is a small-batch training step, and does it capture into a HIP graph?
BERT-large forward + backward (no optimizer) at batch B, eager vs torch.cuda.CUDAGraph replay
(stream capture = hipStreamBeginCapture / hipGraphLaunch on ROCm).

    python scripts/graph_probe.py [--batch 8] [--iters 20]
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
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--seq", type=int, default=512)
    a = ap.parse_args()
    from easydl_amd.models.bert import BERT_LARGE, BertMLM, SyntheticMLM
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = BertMLM(BERT_LARGE, device=dev)
    ids, labels = SyntheticMLM(BERT_LARGE.vocab_size, a.seq).batch(range(a.batch))
    ids, labels = ids.to(dev), labels.to(dev)

    def step():
        loss = m(ids, labels)
        loss.backward()
        return loss

    for p in m.parameters():
        p.grad = torch.zeros_like(p)
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        for _ in range(3):
            step()
    torch.cuda.current_stream(dev).wait_stream(s)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(a.iters):
        step()
    torch.cuda.synchronize(dev)
    eager = (time.perf_counter() - t0) / a.iters
    out = {"batch": a.batch, "eager_ms": round(eager * 1e3, 3)}
    try:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            static_loss = step()
        torch.cuda.synchronize(dev)
        g.replay()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(a.iters):
            g.replay()
        torch.cuda.synchronize(dev)
        graph = (time.perf_counter() - t0) / a.iters
        out.update(graph_ms=round(graph * 1e3, 3), speedup=round(eager / graph, 3),
                   loss=round(float(static_loss), 4))
    except Exception as e:  # noqa: BLE001
        out["graph_error"] = f"{type(e).__name__}: {str(e)[:400]}"
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
