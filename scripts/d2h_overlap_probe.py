"""Does an asynchronous D2H snapshot copy disturb compute?  (The in-memory
checkpoint trace showed the copies running as __amd_rocclr_copyBuffer blit
KERNELS on CUs, not on SDMA engines, and the step time doubling.)

Runs bf16 GEMMs on the compute stream while 8 GB of device memory is copied
in 256 MB chunks into page-locked host memory on a side stream, per mode:
  side        low-priority side stream (what the snapshot engine did)
  cumask<N>   side stream restricted to N CUs (hipExtStreamCreateWithCUMask)
and prints GEMM TFLOP/s alone / with copies and the copy GB/s.
    python scripts/d2h_overlap_probe.py [modes...]
"""
import ctypes
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def cumask_stream(dev, ncu):
    from easydl_amd import _native
    from easydl_amd.operator.reconciler import cu_mask_hex
    from easydl_amd.utils.resources import mask_words
    words = mask_words(cu_mask_hex(ncu))
    arr = (ctypes.c_uint32 * len(words))(*words)
    h = _native.runtime()("edl_stream_create_cumask", dev.index or 0, arr, len(words), 0)
    return torch.cuda.ExternalStream(h, device=dev)


def main():
    dev = torch.device("cuda", 0)
    modes = sys.argv[1:] or ["side", "cumask16", "cumask32"]
    n = 8 << 30
    src = torch.empty(n, dtype=torch.uint8, device=dev).fill_(1)
    dst = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    a = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
    b = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
    iters = 200
    flop = 2 * 8192 ** 3 * iters
    # compute on a non-blocking pool stream: a CU-masked stream is a BLOCKING stream,
    # which the legacy default stream would implicitly serialise with
    comp = torch.cuda.Stream(dev)

    def gemms():
        with torch.cuda.stream(comp):
            for _ in range(iters):
                torch.mm(a, b)

    gemms()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    gemms()
    torch.cuda.synchronize()
    alone = time.perf_counter() - t0
    out = {"env_HSA_ENABLE_SDMA": os.environ.get("HSA_ENABLE_SDMA"), "gemm_alone_tflops": round(flop / alone / 1e12, 1)}
    for mode in modes:
        if mode == "side":
            s = torch.cuda.Stream(dev, priority=0)
        else:
            s = cumask_stream(dev, int(mode[len("cumask"):]))
        chunk = 256 << 20
        copy_done = torch.cuda.Event(enable_timing=False)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(s):
            for o in range(0, n, chunk):
                dst[o:o + chunk].copy_(src[o:o + chunk], non_blocking=True)
            copy_done.record(s)
        gemms()
        comp.synchronize()
        t_gemm = time.perf_counter() - t0
        copy_done.synchronize()
        t_copy = time.perf_counter() - t0
        out[mode] = {"gemm_tflops_with_copy": round(flop / t_gemm / 1e12, 1),
                     "copy_GBps": round(n / t_copy / 1e9, 1), "copy_s": round(t_copy, 3)}
        # copy alone on this stream
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(s):
            for o in range(0, n, chunk):
                dst[o:o + chunk].copy_(src[o:o + chunk], non_blocking=True)
        s.synchronize()
        out[mode]["copy_alone_GBps"] = round(n / (time.perf_counter() - t0) / 1e9, 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
