"""One rank of the xGMI all-reduce test (all ranks share one GPU: IPC mapping
and the flag protocol are exercised exactly as across GPUs; only the link is local)."""
import datetime
import json
import os
import sys
import threading
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from easydl_amd.parallel.xgmi import XgmiComm  # noqa: E402

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
mode = os.environ.get("XG_MODE", "sum")
torch.cuda.set_device(0)
store = dist.TCPStore("127.0.0.1", int(os.environ["PORT"]), world, rank == 0,
                      timeout=datetime.timedelta(seconds=60))
x = XgmiComm(store, "xg", rank, world, torch.device("cuda", 0), ws_bytes=8 << 20, timeout_s=5.0)
res = {"rank": rank, "ok": True, "errors": []}
if mode == "sum":
    cases = [(torch.float32, 1024, "oneshot"), (torch.bfloat16, 4096, "oneshot"), (torch.float32, 1 << 20, "twoshot"),
             (torch.bfloat16, 3 * (1 << 20) + 64, "twoshot"), (torch.float32, 5 << 20, None)]  # last: > workspace
    for dt, n, algo in cases:
        g = torch.Generator(device="cpu").manual_seed(1000 + rank)
        t = torch.randint(-8, 8, (n,), generator=g).to(dt).cuda()
        exp = torch.zeros(n, dtype=torch.float64)
        for r in range(world):
            gr = torch.Generator(device="cpu").manual_seed(1000 + r)
            exp += torch.randint(-8, 8, (n,), generator=gr).double()
        for _ in range(3):  # repeated rounds reuse both parity buffers
            t2 = t.clone()
            x.all_reduce(t2, algo)
        torch.cuda.synchronize()
        if not torch.equal(t2.double().cpu(), exp):
            res["ok"] = False
            res["errors"].append(f"{dt} n={n} algo={algo}: max err {(t2.double().cpu() - exp).abs().max().item()}")
    res["status"] = x.status()
elif mode == "abort":
    # rank 1 never joins the collective: rank 0's kernel must give up on abort, not hang
    if rank == 0:
        t = torch.ones(4096, device="cuda")
        threading.Timer(1.0, x.abort).start()
        t0 = time.time()
        x.all_reduce(t, "oneshot")
        torch.cuda.synchronize()
        res["elapsed"] = time.time() - t0
        res["status"] = x.status()
    store.set(f"done{rank}", "1")
    store.wait([f"done{r}" for r in range(world)])
print(json.dumps(res), flush=True)
with open(os.environ["OUT"] + f".{rank}", "w") as f:
    json.dump(res, f)
x.close()
