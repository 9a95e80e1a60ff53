"""Communication policy and state transfer on the CPU tier (gloo, 2-4 ranks).

* ``Communicator._probe_xgmi``: the per-size RCCL-vs-engine table and the
  selection rule (every decision agreed over the control plane), driven with a
  stand-in engine whose speed the test controls;
* ``Communicator.transfer_state``: multi-source state transfer to joiners,
  slice k from holder k, bit-exact on every receiver.
"""
import datetime
import socket
import threading
import time

import pytest
import torch
import torch.distributed as dist

from easydl_amd.parallel.comm import Communicator


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _spawn(world, fn):
    port = _port()
    out, errs = {}, {}

    def run(r):
        try:
            st = dist.TCPStore("127.0.0.1", port, world, r == 0, timeout=datetime.timedelta(seconds=30))
            c = Communicator(st, r, world, 1, device=torch.device("cpu"), job="pol", timeout_s=20,
                             control_timeout_s=20)
            out[r] = fn(c, st)
        except Exception as e:  # noqa: BLE001
            errs[r] = repr(e)

    ts = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    [t.start() for t in ts]
    [t.join(90) for t in ts]
    assert not errs, errs
    assert len(out) == world
    return out


class FakeEngine:
    """Stands in for XgmiComm: sums over its own gloo group; ``delay(nbytes)`` sets its speed."""

    def __init__(self, comm, delay, broken=False):
        self.c, self.delay, self.broken = comm, delay, broken
        self.timeout_s = 60.0
        self.registered, self.closed, self.calls = [], False, 0

    def register(self, t):
        self.registered.append(t)
        return t

    def unregister(self, r):
        self.registered.remove(r)

    def _find_registered(self, t):
        return None, 0

    def registrable(self, t):
        return True

    def all_reduce(self, t, algo=None):
        if not self.calls:   # the exactness check: a real sum (then only the timing matters)
            self.c.data.allreduce([t]).wait()
            if self.broken:
                t.add_(1)
        self.calls += 1
        time.sleep(self.delay(t.numel() * t.element_size()))
        return t

    def status(self):
        return 0

    def supports(self, t):
        return True

    def close(self):
        self.closed = True


@pytest.mark.parametrize("case", ["engine_wins_large", "engine_loses", "engine_inexact"])
def test_probe_selects_per_size(case):
    def fn(c, st):
        # the "RCCL" side is gloo here: its time is tiny; the engine sleeps per size
        if case == "engine_wins_large":
            delay = lambda nb: 0.0 if nb > (3 << 20) else 0.2  # noqa: E731
        else:
            delay = lambda nb: 0.2  # noqa: E731
        eng = FakeEngine(c, delay, broken=(case == "engine_inexact" and c.rank == 1))
        c.xgmi, c.xgmi_mode = eng, "auto"
        c._probe_xgmi(sizes_mb=(2, 4, 8), iters=1)
        return c.xgmi_probe, c.xgmi_mode, c.xgmi_min_bytes, eng.closed, len(eng.registered)

    out = _spawn(2, fn)
    for probe, mode, min_bytes, closed, nreg in out.values():
        assert nreg == 0                       # the probe buffer is unregistered again
        if case == "engine_wins_large":
            assert probe["selected"] == "xgmi" and mode == "xgmi", probe
            assert probe["xgmi_min_mb_inplace"] == 4 and probe["xgmi_min_mb_staged"] == 4 and min_bytes == 4 << 20
        else:
            assert probe["selected"] == "rccl" and mode is None and closed, probe
        if case == "engine_inexact":
            assert not probe["exact_everywhere"] and probe["sizes_mb"] == []
    assert out[0][0]["selected"] == out[1][0]["selected"]   # agreed, not per rank


@pytest.mark.parametrize("world,holders", [(3, [0, 1]), (4, [1, 3]), (4, [2]), (2, [0, 1])])
def test_transfer_state_multi_source(world, holders):
    def mk(seed, n, dt):
        return torch.randint(-100, 100, (n,), generator=torch.Generator().manual_seed(seed)).to(dt)

    specs = [(1, 1000, torch.float32), (2, 37, torch.float32), (3, 5, torch.int64), (4, 8192, torch.bfloat16)]

    def fn(c, st):
        ts = [mk(seed, n, dt) if c.rank in holders else torch.zeros(n, dtype=dt) for seed, n, dt in specs]
        c.transfer_state(ts, holders)
        return all(torch.equal(t, mk(seed, n, dt)) for t, (seed, n, dt) in zip(ts, specs))

    assert all(_spawn(world, fn).values())
