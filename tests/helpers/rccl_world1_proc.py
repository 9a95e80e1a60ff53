"""The RCCL data plane of ``Communicator`` on real hardware at world 1 (RCCL refuses two
ranks on one GPU): non-blocking communicator init (an epoch aborted while its init may still be
in progress, then a fresh one), every collective the trainer calls, plus the coalesced
point-to-point batch of the multi-source state transfer (a send to and a receive from this rank
in one grouped launch).  Prints one JSON line."""
import datetime
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from easydl_amd.parallel.comm import Communicator  # noqa: E402

os.environ.setdefault("EDL_RCCL_NONBLOCKING", "1")     # (default "auto": re-formed epochs only)
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
store = dist.TCPStore("127.0.0.1", 0, 1, True, timeout=datetime.timedelta(seconds=60))
# an epoch aborted while its non-blocking RCCL init may still be in progress: abort returns
c0 = Communicator(store, 0, 1, 0, device=dev, job="rccl1", timeout_s=60.0, data_backend="auto")
res0 = {"nonblocking": c0.nonblocking}
c0.abort()
c = Communicator(store, 0, 1, 1, device=dev, job="rccl1", timeout_s=60.0, data_backend="auto")
res = {"data_kind": c.data_kind, "backend": c.backend, "nonblocking": c.nonblocking and res0["nonblocking"],
       "aborted_during_init": c0.aborted}
c.warmup()
x = torch.arange(1 << 20, device=dev, dtype=torch.float32)
res["all_reduce"] = bool(torch.equal(c.all_reduce(x.clone()), x))
res["broadcast"] = bool(torch.equal(c.broadcast(x.clone(), 0), x))
out = torch.empty_like(x)
res["all_gather"] = bool(torch.equal(c.all_gather_into(out, x), x))
res["reduce_scatter"] = bool(torch.equal(c.reduce_scatter_into(torch.empty_like(x), x), x))
res["all_to_all"] = bool(torch.equal(c.all_to_all_single(torch.empty_like(x), x), x))
got = torch.zeros_like(x)
c._p2p_batch([("send", x, 0, 0), ("recv", got, 0, 0)])
torch.cuda.current_stream(dev).synchronize()
res["p2p_batch"] = bool(torch.equal(got, x))
c.shutdown()
print(json.dumps(res), flush=True)
