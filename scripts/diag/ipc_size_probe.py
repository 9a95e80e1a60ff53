"""Probe: does hipIpcOpenMemHandle hang for large buffers / several ranks on ONE GPU?
Spawns `ranks` processes per case; each allocates `mb` MiB (torch caching allocator, or
raw hipMalloc via the xGMI workspace when kind=ws) and registers it with every peer
(XgmiComm.register).  Every case runs under its own timeout; prints one JSON line per case."""
import datetime
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def worker():
    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    from easydl_amd.parallel.xgmi import XgmiComm
    rank, world, mb = int(os.environ["RANK"]), int(os.environ["WORLD"]), int(os.environ["MB"])
    torch.cuda.set_device(0)
    st = dist.TCPStore("127.0.0.1", int(os.environ["PORT"]), world, rank == 0, timeout=datetime.timedelta(seconds=60))
    x = XgmiComm(st, "p", rank, world, torch.device("cuda", 0), ws_bytes=16 << 20, timeout_s=20.0)
    extra = [torch.empty(int(os.environ.get("PAD_MB", 0)) << 20, dtype=torch.uint8, device="cuda")]
    buf = torch.zeros((mb << 20) // 2, dtype=torch.bfloat16, device="cuda")
    t0 = time.time()
    x.register(buf)
    t1 = time.time()
    x.all_reduce(buf[: (64 << 20) // 2], "inplace")
    torch.cuda.synchronize()
    print(json.dumps({"rank": rank, "register_s": round(t1 - t0, 3), "status": x.status()}), flush=True)
    st.set(f"d{rank}", "1")
    st.wait([f"d{r}" for r in range(world)])
    del extra
    x.close()


def main():
    cases = [tuple(int(x) for x in c.split(":")) for c in
             os.environ.get("PROBE_CASES", "4:128:0,4:1024:0,2:3900:0,4:3900:0").split(",")]
    for world, mb, pad in cases:
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        env = dict(os.environ, WORLD=str(world), MB=str(mb), PAD_MB=str(pad), PORT=str(port), PYTHONPATH=ROOT)
        t0 = time.time()
        ps = [subprocess.Popen([sys.executable, __file__, "--worker"], env=dict(env, RANK=str(r)),
                               stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True) for r in range(world)]
        outs, ok = [], True
        for p in ps:
            try:
                outs.append(p.communicate(timeout=max(5, 90 - (time.time() - t0)))[0].strip())
            except subprocess.TimeoutExpired:
                ok = False
        for p in ps:
            if p.poll() is None:
                p.kill()
                p.wait()
        print(json.dumps({"ranks": world, "mb": mb, "pad_mb": pad, "completed": ok, "s": round(time.time() - t0, 1),
                          "out": outs}), flush=True)
        if not ok:
            break   # a hung IPC open: stop here, the box has told us enough


if __name__ == "__main__":
    worker() if "--worker" in sys.argv else main()
