"""Child of tests/test_vram_handoff.py: build flat state on the GPU, fill it with 3.0, export it
(utils/vram.publish) and exit once the parent has imported it."""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from easydl_amd.master.store import KV  # noqa: E402
from easydl_amd.optim import FlatAdamW  # noqa: E402
from easydl_amd.parallel.flat import FlatParams  # noqa: E402
from easydl_amd.utils import vram  # noqa: E402

store = dist.TCPStore("127.0.0.1", int(os.environ["VT_PORT"]), is_master=False)
kv = KV(store, "edl/vramtest")
torch.manual_seed(5)
m = torch.nn.Sequential(torch.nn.Linear(256, 512), torch.nn.Linear(512, 256)).to("cuda", torch.bfloat16)
f = FlatParams(m)
o = FlatAdamW(f)
ts = {}
for g in f.groups:
    ts[f"flat/{g.name}/data"], ts[f"flat/{g.name}/grad"] = g.data, g.grad
for g, st in zip(f.groups, o.state):
    for k, t in st.items():
        if isinstance(t, torch.Tensor) and t is not g.data:
            ts[f"opt/{g.name}/{k}"] = t
for t in ts.values():
    t.fill_(3.0)
torch.cuda.synchronize()
n = vram.publish(kv, "worker0", "vt-child", ts)
assert n == len(ts), (n, len(ts))
kv.set("vt/published", "1")
assert kv.wait_for("vt/imported", 120)
sys.exit(0)
