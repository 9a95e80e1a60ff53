"""One rank of the Communicator(data_backend="xgmi") test: ElasticDDP-style
bucket all-reduces go through the xGMI engine's async path (its own stream,
event-ordered), and a give-up is reported by healthy().  All ranks share one
GPU, so no RCCL collective is issued (RCCL refuses two ranks on one device)."""
import datetime
import json
import os
import sys
import threading
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from easydl_amd.parallel.comm import Communicator  # noqa: E402

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
mode = os.environ.get("XG_MODE", "sum")
torch.cuda.set_device(0)
store = dist.TCPStore("127.0.0.1", int(os.environ["PORT"]), world, rank == 0,
                      timeout=datetime.timedelta(seconds=60))
# barriers give up 5 s after entry in the abort test; elsewhere host-side verification
# between iterations must never look like a dead peer (and ranks meet at a store barrier)
c = Communicator(store, rank, world, 3, device=torch.device("cuda", 0), job="t",
                 timeout_s=float(os.environ.get("XG_TIMEOUT", 5.0 if mode == "abort" else 30.0)), data_backend="xgmi")
NOSYNC = os.environ.get("XG_NOSYNC") == "1"   # diagnostics: round-2 behaviour (no store barrier)
res = {"rank": rank, "ok": True, "errors": [], "backend": c.backend}
_n = [0]


def sync():
    res.setdefault("t_launch", []).append(round(time.time(), 4))
    if NOSYNC:
        return
    _n[0] += 1
    store.set(f"it{_n[0]}/{rank}", "1")
    store.wait([f"it{_n[0]}/{r}" for r in range(world)])


if mode == "sum":
    grads = torch.empty(3 * (1 << 20) + 4096, device="cuda", dtype=torch.bfloat16)
    buckets = [grads[:4096], grads[4096:4096 + (1 << 20)], grads[4096 + (1 << 20):]]
    for it in range(3):
        g = torch.Generator(device="cpu").manual_seed(100 * it + rank)
        grads.copy_(torch.randint(-8, 8, grads.shape, generator=g).to(torch.bfloat16))
        exp = torch.zeros(grads.numel(), dtype=torch.float64)
        for r in range(world):
            exp += torch.randint(-8, 8, grads.shape, generator=torch.Generator().manual_seed(100 * it + r)).double()
        sync()
        works = [c.all_reduce_async(b) for b in buckets]  # issued in bucket order, overlapping
        for w in works:
            w.wait()
        torch.cuda.current_stream().synchronize()
        if not torch.equal(grads.double().cpu(), exp):
            res["ok"] = False
            res["errors"].append(f"iter {it}: max err {(grads.double().cpu() - exp).abs().max().item()}")
    res["healthy"] = c.healthy()
elif mode == "coll":
    # TP / SP collectives on the engine: integer-valued data, so results are exact
    def ints(shape, seed, dtype):
        return torch.randint(-64, 64, shape, generator=torch.Generator().manual_seed(seed)).to(dtype)
    for dtype in (torch.float32, torch.bfloat16):
        n = 3 * 4096 + 64
        t = ints((n,), 7 + rank, dtype).cuda()
        exp = torch.stack([ints((n,), 7 + r, dtype) for r in range(world)]).float().amax(0)
        c.all_reduce(t, dist.ReduceOp.MAX)
        if not torch.equal(t.float().cpu(), exp):
            res["ok"] = False
            res["errors"].append(f"max {dtype}")
        # all-gather / reduce-scatter, one message that needs several workspace pieces (64 MiB)
        m = (24 << 20) // torch.tensor([], dtype=dtype).element_size() + 256
        inp = ints((m,), 11 + rank, dtype).cuda()
        out = torch.empty(world * m, dtype=dtype, device="cuda")
        c.all_gather_into(out, inp)
        exp = torch.cat([ints((m,), 11 + r, dtype) for r in range(world)])
        if not torch.equal(out.cpu(), exp):
            res["ok"] = False
            res["errors"].append(f"all_gather {dtype}")
        big = ints((world * m,), 13 + rank, dtype).cuda()
        part = torch.empty(m, dtype=dtype, device="cuda")
        c.reduce_scatter_into(part, big)
        exp = sum(ints((world * m,), 13 + r, dtype).double() for r in range(world))[rank * m:(rank + 1) * m]
        if not torch.equal(part.double().cpu(), exp):
            res["ok"] = False
            res["errors"].append(f"reduce_scatter {dtype}: max err {(part.double().cpu() - exp).abs().max().item()}")
    torch.cuda.synchronize()
    res["healthy"] = c.healthy()
elif mode == "mixed":
    # async bucket all-reduces still pending on the engine stream while sync collectives
    # are issued on the SAME comm from the caller's stream: they must queue behind them
    x = c.xgmi
    for it in range(3):
        def ints(n, seed):
            return torch.randint(-32, 32, (n,), generator=torch.Generator().manual_seed(seed)).float()
        big = [ints(6 << 20, 1000 * it + 10 * k + rank).cuda() for k in range(3)]
        m = 5 << 20
        inp = ints(world * m, 2000 * it + rank).cuda()
        sync()
        works = [x.all_reduce_async(b) for b in big]
        part = torch.empty(m, device="cuda")
        x.reduce_scatter(part, inp)
        gat = torch.empty(world * m, device="cuda")
        x.all_gather(gat, part)
        for w in works:
            w.wait()
        torch.cuda.synchronize()
        for k, b in enumerate(big):
            exp = sum(ints(6 << 20, 1000 * it + 10 * k + r) for r in range(world))
            if not torch.equal(b.cpu(), exp):
                res["ok"] = False
                res["errors"].append(f"iter {it} bucket {k}")
        red = sum(ints(world * m, 2000 * it + r) for r in range(world))
        if not torch.equal(part.cpu(), red[rank * m:(rank + 1) * m]) or not torch.equal(gat.cpu(), red):
            res["ok"] = False
            res["errors"].append(f"iter {it} rs/ag")
    res["healthy"] = c.healthy()
    res["detail"] = x.status_detail()
elif mode == "abort":
    if rank == 0:  # the peer never joins: the watchdog's abort() releases the kernel, healthy() says so
        t = torch.ones(1 << 16, device="cuda", dtype=torch.bfloat16)
        threading.Timer(1.0, c.abort).start()
        w = c.all_reduce_async(t)
        w.wait()
        torch.cuda.synchronize()
        res["healthy"] = c.healthy()
        res["aborted"] = c.aborted
    store.set(f"done{rank}", "1")
    store.wait([f"done{r}" for r in range(world)])
if c.xgmi is not None and "detail" not in res:
    res["detail"] = c.xgmi.status_detail()
print(json.dumps(res), flush=True)
with open(os.environ["OUT"] + f".{rank}", "w") as f:
    json.dump(res, f)
c.xgmi.close()
