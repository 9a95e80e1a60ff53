"""Native RCCL communicator manager (csrc/runtime/rccl_comm.cpp) on one GPU.

Multi-rank collectives need several GPUs (RCCL refuses two ranks on one
device); here: the library resolves against torch's RCCL, world-1 collectives
are exact, and — the point of the non-blocking design — creating a 2-rank
communicator whose peer never arrives is abandoned promptly by abort()."""
import datetime
import socket
import threading
import time

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


def _store():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return dist.TCPStore("127.0.0.1", port, 1, True, timeout=datetime.timedelta(seconds=30))


def test_rccl_resolves(cuda):
    from easydl_amd.parallel import rccl
    ok, ver, _ = rccl.available()
    assert ok and ver > 0


def test_world1_collectives_native(cuda):
    from easydl_amd.parallel.comm import Communicator
    c = Communicator(_store(), 0, 1, 1, device=torch.device("cuda", 0), data_backend="native")
    assert c.backend == "rccl-native"
    c.warmup()
    x = torch.arange(1000, device="cuda", dtype=torch.float32)
    c.all_reduce(x)
    y = torch.randn(4096, device="cuda", dtype=torch.bfloat16)
    y0 = y.clone()
    c.broadcast(y, 0)
    out = torch.empty(4096, device="cuda", dtype=torch.bfloat16)
    c.all_gather_into(out, y)
    rs = torch.empty(4096, device="cuda", dtype=torch.bfloat16)
    c.reduce_scatter_into(rs, y)
    w = c.all_reduce_async(x)
    w.wait()
    torch.cuda.synchronize()
    assert torch.equal(x, torch.arange(1000, device="cuda", dtype=torch.float32))
    assert torch.equal(y, y0) and torch.equal(out, y0) and torch.equal(rs, y0)
    c.shutdown()


@pytest.mark.timeout(90)
def test_pending_init_is_abortable(cuda):
    """Rank 0 of a 2-rank communicator whose peer never comes: abort() ends the wait."""
    from easydl_amd.parallel.rccl import RcclComm, RcclError
    store = _store()
    box = {}

    def build():
        try:
            RcclComm(store, "t", 0, 2, torch.device("cuda", 0), timeout_s=60)
        except RcclError as e:
            box["err"] = str(e)

    holder = {}
    orig_init = RcclComm.__init__

    def spy(self, *a, **k):
        holder["c"] = self
        orig_init(self, *a, **k)

    RcclComm.__init__ = spy
    try:
        th = threading.Thread(target=build)
        t0 = time.time()
        th.start()
        time.sleep(1.0)
        holder["c"].abort()
        th.join(20)
    finally:
        RcclComm.__init__ = orig_init
    assert not th.is_alive(), "init did not return after abort"
    assert "aborted" in box.get("err", ""), box
    assert time.time() - t0 < 15
