"""Who holds GPU memory after a standby's full-width warm-up?  Runs warm_device three
times, then lists the live CUDA tensors Python can see and what refers to them."""
import gc
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from easydl_amd.operator.standby import warm_device  # noqa: E402

spec = {"model": "llama", "batch": [1, 512],
        "cfg": {"vocab_size": 4096, "dim": 1024, "n_layers": 4, "n_heads": 8, "n_kv_heads": 2, "ffn_dim": 2048,
                "max_seq_len": 512}}
mem = []
for _ in range(3):
    warm_device(0, spec)
    torch.cuda.synchronize()
    gc.collect()
    mem.append(torch.cuda.memory_allocated(0) >> 20)
print(json.dumps({"allocated_mb": mem}), flush=True)
live = []
for o in gc.get_objects():
    try:
        if isinstance(o, torch.Tensor) and o.is_cuda:
            live.append(o)
    except Exception:  # noqa: BLE001
        pass
live.sort(key=lambda t: -t.untyped_storage().nbytes())
print("live cuda tensors:", len(live), "storage MB total (may double count views):",
      sum(t.untyped_storage().nbytes() for t in live) >> 20)
seen = set()
for t in live[:12]:
    st = t.untyped_storage().data_ptr()
    if st in seen:
        continue
    seen.add(st)
    refs = [type(r).__name__ + (f":{list(r.keys())[:6]}" if isinstance(r, dict) else "") for r in gc.get_referrers(t)
            if r is not live]
    print(f"{tuple(t.shape)} {t.dtype} storage={t.untyped_storage().nbytes() >> 20}MB "
          f"param={isinstance(t, torch.nn.Parameter)} refs={refs[:6]}", flush=True)
    for r in gc.get_referrers(t):
        if isinstance(r, dict) and r is not live:
            owners = [type(x).__name__ for x in gc.get_referrers(r) if x is not live][:6]
            print("   dict owner:", owners, flush=True)
