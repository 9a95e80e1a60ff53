"""H2D restore bandwidth from a /dev/shm snapshot slot, as a replacement worker
sees it (fresh process, the segment's pages never mapped in it before).

    python scripts/restore_bench.py --gb 24            # writer, then one fresh process per method

Method: ``pipelined`` (multi-threaded memcpy into pinned staging + DMA) — the
restore path of easydl_amd/ckpt/manager.py.  (A zero-copy variant that
hipHostRegister-ed windows of the slot in place measured 12 GB/s vs 36-44 GB/s
for this one on MI355X: pinning pages costs more than the staging copy.)
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

NAME = "/edl-restorebench"


def writer(gb: float) -> None:
    from easydl_amd.ckpt.manager import ShmSegment
    n = int(gb * (1 << 30))
    seg = ShmSegment(NAME, n, create=True, pin=False)
    slot = seg.begin()
    v = seg.view(slot, 0, n)
    step = 64 << 20
    for o in range(0, n, step):
        v[o:o + step] = (o // step) % 251 + 1
    seg.commit(slot, 1, 1, n, 0, {})
    seg.close()


def reader(method: str, gb: float) -> dict:
    import torch

    from easydl_amd import _native
    from easydl_amd.ckpt.manager import ShmSegment
    n = int(gb * (1 << 30))
    dev = torch.device("cuda", 0)
    dst = torch.empty(n, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    seg = ShmSegment(NAME, create=False)
    slot = seg.committed()[0]["slot"]
    parts = 8  # like a state table: several tensors
    per = n // parts
    arr = lambda v: (ctypes.c_uint64 * parts)(*v)  # noqa: E731
    ptrs = arr([dst.data_ptr() + i * per for i in range(parts)])
    sizes = arr([per] * parts)
    offs = arr([i * per for i in range(parts)])
    stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    t0 = time.perf_counter()
    rc = _native.runtime()("edl_ckpt_restore_pipelined", seg.h, slot, parts, ptrs, sizes, offs, stream,
                           256 << 20, 16)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ok = rc == 0 and bool((dst[:4096].cpu().numpy() == seg.view(slot, 0, 4096)).all())
    seg.close()
    return {"method": method, "gb": gb, "s": round(dt, 3), "GBps": round(n / dt / 1e9, 2), "rc": rc, "ok": ok}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gb", type=float, default=24.0)
    ap.add_argument("--role", default="driver")
    ap.add_argument("--method", default="")
    a = ap.parse_args()
    if a.role == "writer":
        return writer(a.gb)
    if a.role == "reader":
        print(json.dumps(reader(a.method, a.gb)), flush=True)
        return
    try:
        subprocess.run([sys.executable, __file__, "--role", "writer", "--gb", str(a.gb)], check=True)
        for m in ("pipelined", "pipelined"):
            subprocess.run([sys.executable, __file__, "--role", "reader", "--method", m, "--gb", str(a.gb)],
                           check=True, timeout=300)
    finally:
        try:
            os.unlink("/dev/shm" + NAME)
        except OSError:
            pass


if __name__ == "__main__":
    main()
