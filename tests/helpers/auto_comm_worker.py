"""One rank of the default "auto" data-plane test on ONE GPU shared by 2-4 ranks.

The real xGMI engine (csrc/kernels/xgmi.hip) goes through the whole path the
8-GPU job takes: ``warmup()`` -> ``_probe_xgmi`` (timed in the training form:
``all_reduce_async`` at ``async_blocks`` workgroups) -> policy agreed and cached
per (group, world) -> ``ElasticDDP.set_comm`` registers the flat gradient buffers
-> one DDP step whose bucket all-reduces run on the engine, overlapped with the
backward.  gloo on GPU tensors stands in for RCCL (RCCL refuses two ranks on one
device).  A second epoch of the same world then adopts the cached policy
without timing anything (the re-formation path)."""
import datetime
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from easydl_amd.models.mlp import MLP  # noqa: E402
from easydl_amd.parallel.comm import Communicator  # noqa: E402
from easydl_amd.parallel.ddp import ElasticDDP  # noqa: E402
from easydl_amd.parallel.flat import FlatParams  # noqa: E402

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
store = dist.TCPStore("127.0.0.1", int(os.environ["PORT"]), world, rank == 0,
                      timeout=datetime.timedelta(seconds=90))
res = {"rank": rank, "ok": True, "errors": []}

# the engine must win somewhere against the gloo stand-in (it does by a wide margin: gloo
# stages GPU tensors through the host), so the policy routes the registered buffers to it
c = Communicator(store, rank, world, 1, device=dev, job="auto", timeout_s=60.0, data_backend="auto-gloo",
                 probe="now")
t0 = time.perf_counter()
c.warmup()
res["warmup_s"] = round(time.perf_counter() - t0, 3)
res["probe"] = c.xgmi_probe
res["backend"] = c.backend

torch.manual_seed(0)   # identical replicas
model = MLP(784, (1024, 1024), 10, device=dev, dtype=torch.float32)
flat = FlatParams(model)
ddp = ElasticDDP(flat, None, bucket_mb=1.0)     # several buckets -> several async all-reduces
ddp.set_comm(c)
res["registered"] = len(c.xgmi._registered) if c.xgmi is not None else 0
res["buckets"] = len(ddp.buckets)

g = torch.Generator().manual_seed(100 + rank)
x = torch.randn(64, 784, generator=g).to(dev)
y = torch.randint(0, 10, (64,), generator=g).to(dev)

# local gradient (no communication) -> reference sum over the control plane (fp64, host)
flat.zero_grad()
with ddp.no_sync():
    model(x, y).backward()
flat.finalize_untouched()
local = torch.cat([gr.grad.detach().double().cpu().reshape(-1) for gr in flat.groups])
ref = local.clone()
dist_ref = c.ctrl_all_reduce(ref.numpy(), dist.ReduceOp.SUM)   # float64 sum over ranks

# the DDP step proper: buckets all-reduced by the engine under the backward
flat.zero_grad()
ddp.prepare()
model(x, y).backward()
ddp.finish()
torch.cuda.current_stream().synchronize()
got = torch.cat([gr.grad.detach().double().cpu().reshape(-1) for gr in flat.groups])
err = (got - dist_ref).abs().max().item()
scale = dist_ref.abs().max().item()
res["max_rel_err"] = err / max(scale, 1e-30)
if not (err <= 1e-5 * max(scale, 1.0)):
    res["ok"] = False
    res["errors"].append(f"ddp grad mismatch: max abs err {err} (scale {scale})")
res["healthy"] = c.healthy()
res["status"] = c.xgmi.status() if c.xgmi is not None else None
c.barrier()
c.shutdown()

# epoch 2 of the same world (a re-formation): the cached policy, nothing timed
c2 = Communicator(store, rank, world, 2, device=dev, job="auto", timeout_s=60.0, data_backend="auto-gloo",
                  probe="defer")
t0 = time.perf_counter()
c2.warmup()
res["warmup2_s"] = round(time.perf_counter() - t0, 3)
res["probe2"] = c2.xgmi_probe
res["pending2"] = c2.probe_pending
res["backend2"] = c2.backend
c2.barrier()
c2.shutdown()
with open(f"{os.environ['OUT']}.{rank}", "w") as f:
    json.dump(res, f, default=str)
