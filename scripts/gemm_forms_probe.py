"""Can the SwiGLU MLP drop one of its two activation copies?  The fused kernels write
both h and h^T (forward) and both d(gate_up) and d(gate_up)^T (backward); each GEMM
reads one of them.  This times every GEMM of the MLP in the form it has now and in the
form that would read the OTHER copy (M = 16384 tokens, D 4096, F 14336):

  down.fwd     y = h @ Wd^T         now: mm(h, Wd.t())          alt: mm(hT.t(), Wd.t())
  gu.dgrad     dx = dgu @ Wgu       now: mm(dgu, WguT.t())      alt: mm(dguT.t(), WguT.t()), mm(dguT.t(), Wgu)

One JSON line per form."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=15):
    for _ in range(4):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    dev = torch.device("cuda")
    M, D, F = 16384, 4096, 14336
    g = torch.Generator(device=dev).manual_seed(0)
    rnd = lambda *s: torch.randn(*s, device=dev, generator=g).to(torch.bfloat16)  # noqa: E731
    h = rnd(M, F)
    hT = h.t().contiguous()
    wd = rnd(D, F) * 0.02
    dgu = rnd(M, 2 * F)
    dguT = dgu.t().contiguous()
    wgu = rnd(2 * F, D) * 0.02
    wguT = wgu.t().contiguous()
    forms = {
        "down.fwd now mm(h, Wd.t())": (lambda: torch.mm(h, wd.t()), 2.0 * M * F * D),
        "down.fwd alt mm(hT.t(), Wd.t())": (lambda: torch.mm(hT.t(), wd.t()), 2.0 * M * F * D),
        "gu.dgrad now mm(dgu, WguT.t())": (lambda: torch.mm(dgu, wguT.t()), 2.0 * M * 2 * F * D),
        "gu.dgrad alt mm(dguT.t(), WguT.t())": (lambda: torch.mm(dguT.t(), wguT.t()), 2.0 * M * 2 * F * D),
        "gu.dgrad alt mm(dguT.t(), Wgu)": (lambda: torch.mm(dguT.t(), wgu), 2.0 * M * 2 * F * D),
    }
    ref = {}
    for name, (fn, flops) in forms.items():
        t = timeit(fn)
        out = fn()
        key = name.split()[0]
        err = None
        if key in ref:
            err = ((out.float() - ref[key]).abs().max() / ref[key].abs().max()).item()
        else:
            ref[key] = out.float()
        print(json.dumps({"form": name, "ms": round(t * 1e3, 3), "tflops": round(flops / t / 1e12, 1),
                          "rel_err_vs_now": err}), flush=True)


if __name__ == "__main__":
    main()
