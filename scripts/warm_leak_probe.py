"""Which cache keeps GPU memory after a standby's full-width warm-up (operator/standby.py)?
Prints the growth of torch.cuda.memory_allocated over three warm-up calls in this process."""
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
    mem.append(torch.cuda.memory_allocated(0) >> 20)
print(json.dumps({"env": {k: os.environ.get(k) for k in ("EDL_GEMM_TUNING", "EDL_WT_CACHE")},
                  "allocated_mb": mem}), flush=True)
