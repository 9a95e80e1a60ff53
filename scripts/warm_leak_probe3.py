"""Referrer chains of the FlatParams / Llama objects still alive after standby warm-ups."""
import gc
import os
import sys
import types

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from easydl_amd.operator.standby import warm_device  # noqa: E402
from easydl_amd.parallel.flat import FlatParams  # noqa: E402
from easydl_amd.models.llama import Llama  # noqa: E402

spec = {"model": "llama", "batch": [1, 512],
        "cfg": {"vocab_size": 4096, "dim": 1024, "n_layers": 4, "n_heads": 8, "n_kv_heads": 2, "ffn_dim": 2048,
                "max_seq_len": 512}}
for _ in range(2):
    warm_device(0, spec)
torch.cuda.synchronize()
gc.collect()
print("allocated MB", torch.cuda.memory_allocated(0) >> 20, flush=True)


def describe(o):
    if isinstance(o, types.FrameType):
        return f"frame {o.f_code.co_name} {o.f_code.co_filename}:{o.f_lineno}"
    if isinstance(o, types.FunctionType):
        return f"function {o.__qualname__} ({o.__module__})"
    if isinstance(o, types.MethodType):
        return f"method {o.__func__.__qualname__}"
    if isinstance(o, types.CellType):
        return "cell"
    if isinstance(o, dict):
        return f"dict keys={list(o.keys())[:5]}"
    if isinstance(o, (list, tuple)):
        return f"{type(o).__name__} len={len(o)}"
    return type(o).__module__ + "." + type(o).__qualname__


def chain(obj, depth=0, seen=None, maxd=6):
    seen = seen if seen is not None else set()
    if depth > maxd:
        return
    for r in gc.get_referrers(obj):
        if id(r) in seen or r is sys._getframe() or isinstance(r, types.FrameType) and r.f_code.co_name == "chain":
            continue
        seen.add(id(r))
        print("  " * depth + "<- " + describe(r), flush=True)
        if isinstance(r, types.ModuleType):
            continue
        chain(r, depth + 1, seen, maxd)


objs = [o for o in gc.get_objects() if isinstance(o, (FlatParams, Llama))]
print("alive:", [type(o).__name__ for o in objs], flush=True)
for o in objs[:2]:
    print("==", type(o).__name__, flush=True)
    chain(o, maxd=5)
