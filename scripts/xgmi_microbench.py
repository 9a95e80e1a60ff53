#!/usr/bin/env python
"""xGMI engine microbenchmark on ONE GPU: N ranks share the device, so every
"peer" access is a local-HBM access through an IPC mapping.  This measures the
engine's kernels (barrier cost, memory-level parallelism, HBM efficiency) —
not xGMI link bandwidth, which needs an 8-GPU node.

Per op and rank, the in-place two-shot all-reduce of S bytes moves
  reduce-scatter: reads S (chunk r from all N ranks) + writes S/N
  all-gather:     reads (N-1)/N S + writes (N-1)/N S
so N ranks together move about 3*N*S bytes of HBM traffic per op; the report
gives that as achieved HBM GB/s next to the algorithmic bus bandwidth.

Usage: python scripts/xgmi_microbench.py --ranks 4 --mb 64 256 --iters 10
"""
from __future__ import annotations

import argparse
import datetime
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def worker():
    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    from easydl_amd.parallel.xgmi import XgmiComm

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    sizes = [float(x) for x in os.environ["XB_MB"].split(",")]
    iters = int(os.environ["XB_ITERS"])
    torch.cuda.set_device(0)
    st = dist.TCPStore("127.0.0.1", int(os.environ["PORT"]), world, rank == 0, timeout=datetime.timedelta(seconds=60))
    x = XgmiComm(st, "xb", rank, world, torch.device("cuda", 0), timeout_s=30.0)
    n = 0

    def sync(tag):
        nonlocal n
        n += 1
        st.set(f"{tag}{n}/{rank}", "1")
        st.wait([f"{tag}{n}/{r}" for r in range(world)])

    buf = torch.ones(int(max(sizes) * (1 << 20)) // 2, dtype=torch.bfloat16, device="cuda")
    reg = x.register(buf)
    res = []
    for mb in sizes:
        view = buf[:int(mb * (1 << 20)) // 2]
        forms = [("inplace", lambda: x.all_reduce(view, "inplace")),
                 ("staged", lambda: x.all_reduce(view, "twoshot")),
                 ("pull", lambda: x.pull([view], [0]))]
        if mb <= 4:
            forms.append(("oneshot", lambda: x.all_reduce(view, "oneshot")))
        for algo, fn in forms:
            fn()
            torch.cuda.synchronize()
            sync("w")
            t0 = time.perf_counter()
            for _ in range(iters):
                fn()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / iters
            sync("e")
            res.append({"mb": mb, "algo": algo, "ms": round(dt * 1e3, 3)})
    if rank == 0:
        from easydl_amd import _native
        print(json.dumps({"rank": rank, "blocks": x.blocks, "res": res, "status": x.status_detail(),
                          "wallclock_hz": _native.kernels()("edl_xgmi_wallclock_hz")}), flush=True)
    sync("z")
    x.unregister(reg)
    x.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, nargs="+", default=[2, 4])
    ap.add_argument("--mb", type=float, nargs="+", default=[16, 128])
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    rows = []
    for world in a.ranks:
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        env = dict(os.environ, WORLD_SIZE=str(world), PORT=str(port), XB_MB=",".join(map(str, a.mb)),
                   XB_ITERS=str(a.iters), PYTHONPATH=ROOT)
        procs = [subprocess.Popen([sys.executable, __file__, "--worker"], env=dict(env, RANK=str(r)),
                                  stdout=subprocess.PIPE, text=True) for r in range(world)]
        outs = [p.communicate(timeout=300)[0] for p in procs]
        if any(p.returncode for p in procs):
            raise SystemExit(f"world {world}: worker failed {[p.returncode for p in procs]}")
        d = json.loads([ln for ln in outs[0].splitlines() if ln.startswith("{")][0])
        for r in d["res"]:
            S = r["mb"] * (1 << 20)
            t = r["ms"] / 1e3
            if r["algo"] == "pull":
                traffic = 2 * (world - 1) * S          # every receiver reads S and writes S
            elif r["algo"] == "oneshot":                # stage copy + every rank reads N x S
                traffic = world * (2 * S + world * S + S)
            elif r["algo"] == "inplace":
                traffic = world * (S + S / world + 2 * (world - 1) / world * S)
            else:                                       # staged: + stage copy (read S, write S)
                traffic = world * (3 * S + S / world + 2 * (world - 1) / world * S)
            row = dict(r, ranks=world, blocks=d["blocks"], wallclock_hz=d["wallclock_hz"],
                       busbw_gbs=round(2 * (world - 1) / world * S / t / 1e9, 1) if r["algo"] != "pull" else None,
                       hbm_gbs=round(traffic / t / 1e9, 1))
            rows.append(row)
            print(json.dumps(row), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    if "--worker" in sys.argv:
        worker()
    else:
        main()
