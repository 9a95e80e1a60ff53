"""One rank of the xGMI engine tests (all ranks share one GPU: IPC mapping and
the flag protocol are exercised exactly as across GPUs; only the link is local).

Ranks meet at a store barrier before every case: the engine's barriers wait
for peers for at most ``timeout_s`` from barrier entry, and the expected values
are computed on the CPU between cases (host skew must not look like a dead peer).
"""
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
x = XgmiComm(store, "xg", rank, world, torch.device("cuda", 0), ws_bytes=8 << 20,
             timeout_s=5.0 if mode == "abort" else 30.0)
res = {"rank": rank, "ok": True, "errors": [], "blocks": x.blocks, "ranks_per_device": x.ranks_per_device}
_n = [0]


def sync():
    _n[0] += 1
    store.set(f"b{_n[0]}/{rank}", "1")
    store.wait([f"b{_n[0]}/{r}" for r in range(world)])


def ints(n, seed, dt):
    return torch.randint(-8, 8, (n,), generator=torch.Generator().manual_seed(seed)).to(dt)


if mode == "sum":
    cases = [(torch.float32, 1024, "oneshot"), (torch.bfloat16, 4096, "oneshot"), (torch.float32, 1 << 20, "twoshot"),
             (torch.bfloat16, 3 * (1 << 20) + 64, "twoshot"), (torch.float32, 5 << 20, None)]  # last: > workspace
    for dt, n, algo in cases:
        t = ints(n, 1000 + rank, dt).cuda()
        exp = sum(ints(n, 1000 + r, dt).double() for r in range(world))
        sync()
        for _ in range(3):  # repeated rounds reuse both parity buffers
            t2 = t.clone()
            x.all_reduce(t2, algo)
        torch.cuda.synchronize()
        if not torch.equal(t2.double().cpu(), exp):
            res["ok"] = False
            res["errors"].append(f"{dt} n={n} algo={algo}: max err {(t2.double().cpu() - exp).abs().max().item()}")
    res["status"] = x.status()
    res["detail"] = x.status_detail()
elif mode == "inplace":
    # registered buffer (the flat-gradient case): bucket slices all-reduced in place,
    # one launch each, several rounds and buckets in flight on the engine stream
    for dt in (torch.bfloat16, torch.float32):
        n = 3 * (1 << 20) + 4096 + 64 * 7   # odd chunking: the last rank's chunk is short
        grads = torch.empty(n, dtype=dt, device="cuda")
        reg = x.register(grads)
        bounds = [0, 4096, 4096 + (1 << 20), n]   # 8 KB bucket: staged one-shot; others in place
        for it in range(3):
            grads.copy_(ints(n, 100 * it + rank, dt).cuda())
            exp = sum(ints(n, 100 * it + r, dt).double() for r in range(world))
            sync()
            works = [x.all_reduce_async(grads[a:b]) for a, b in zip(bounds[:-1], bounds[1:])]
            for w in works:
                w.wait()
            torch.cuda.current_stream().synchronize()
            if not torch.equal(grads.double().cpu(), exp):
                bad = (grads.double().cpu() - exp).abs()
                res["ok"] = False
                res["errors"].append(f"{dt} iter {it}: max err {bad.max().item()} at {int(bad.argmax())}")
        sync()
        x.unregister(reg)
    res["status"] = x.status()
    res["detail"] = x.status_detail()
elif mode == "pull":
    # state transfer: ranks 0..h-1 hold the state, the others receive it from all holders
    holders = list(range(max(1, world // 2)))
    shapes = ((1 << 20, torch.float32), (3 * 4096 + 8, torch.bfloat16), (4 * 1000, torch.int32),
              (6 * (1 << 20) + 4, torch.float32))   # 24 MB: several staged windows of the 8 MB workspace
    ts = [torch.empty(n, dtype=dt, device="cuda") for n, dt in shapes]
    for i, t in enumerate(ts):
        t.copy_(ints(t.numel(), 77 + i, t.dtype).cuda() if rank in holders else torch.zeros_like(t))
    sync()
    t0 = time.time()
    x.pull(ts, holders)
    torch.cuda.synchronize()
    res["elapsed"] = time.time() - t0
    for i, t in enumerate(ts):
        if not torch.equal(t.cpu(), ints(t.numel(), 77 + i, t.dtype)):
            res["ok"] = False
            res["errors"].append(f"tensor {i} differs on rank {rank}")
    res["status"] = x.status()
elif mode == "reglimit":
    # a segment over the mapping limit (EDL_XGMI_REGISTER_MAX_MB) is refused on EVERY rank,
    # before any IPC open, and the tensor still all-reduces (staged)
    x.REGISTER_MAX = 1 << 20
    t = ints(1 << 20, 5 + rank, torch.float32).cuda()    # 4 MB tensor in a >= 4 MB segment
    try:
        x.register(t)
        res["refused"] = False
    except Exception as e:  # noqa: BLE001
        res["refused"] = "exceeds the IPC mapping limit" in str(e)
    sync()
    x.all_reduce(t)
    torch.cuda.synchronize()
    if not torch.equal(t.cpu(), sum(ints(1 << 20, 5 + r, torch.float32) for r in range(world))):
        res["ok"] = False
        res["errors"].append("staged all-reduce after refusal")
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
        res["detail"] = x.status_detail()
        t1 = time.time()
        x.close_after_abort()                # what the trainer does with an aborted epoch's engine
        res["release_s"] = time.time() - t1
        res["released"] = x._ws is None
    store.set(f"done{rank}", "1")
    store.wait([f"done{r}" for r in range(world)])
elif mode == "lifetime":
    # IPC lifetime (docs/design_notes.md): rank 1 registers a buffer and EXITS; rank 0 then
    # copies from its mapping of that buffer.  With dmabuf IPC the import holds a reference
    # on the buffer object, so the memory must still be there with rank 1's data.
    t = torch.full((1 << 20,), float(rank + 7), device="cuda")
    reg = x.register(t)
    torch.cuda.synchronize()
    store.set(f"pid{rank}", str(os.getpid()))
    sync()
    if rank == 1:
        with open(os.environ["OUT"] + f".{rank}", "w") as f:
            json.dump(res, f)
        os._exit(0)
    import ctypes
    pid = int(store.get("pid1"))
    t_end = time.time() + 30
    while time.time() < t_end:
        try:
            state = open(f"/proc/{pid}/stat").read().rsplit(")", 1)[1].split()[0]
        except OSError:
            state = "gone"
        if state in ("Z", "X", "gone"):
            break
        time.sleep(0.05)
    res["exporter_state"] = state
    time.sleep(2.0)    # let the driver finish tearing the dead process down
    out = torch.zeros_like(t)
    hip = ctypes.CDLL("libamdhip64.so")
    rc = hip.hipMemcpy(ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(reg.peers[1]),
                       ctypes.c_size_t(t.numel() * 4), 3)    # hipMemcpyDeviceToDevice
    torch.cuda.synchronize()
    res["rc"] = rc
    res["ok"] = rc == 0 and bool(torch.all(out == 8.0))
    with open(os.environ["OUT"] + f".{rank}", "w") as f:
        json.dump(res, f)
    os._exit(0)
print(json.dumps(res), flush=True)
with open(os.environ["OUT"] + f".{rank}", "w") as f:
    json.dump(res, f)
sync()
x.close()
