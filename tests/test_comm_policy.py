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
        self.registered, self.closed, self.calls, self.gate_calls = [], False, 0, 0

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
        if t.numel() == Communicator.GATE_ELEMS:   # exactness gate of an adopted policy: a real sum
            self.gate_calls += 1
            self.c.data.allreduce([t]).wait()
            if self.broken:
                t.add_(1)
            return t
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


# --- the policy function shared by the per-epoch probe and the Brain ------------------

def test_decide_oneshot_crossover_first_win_and_bucket_knee():
    from easydl_amd.parallel.comm_policy import decide
    inf = float("inf")
    kb = [256, 1024, 4096, 32768, 131072]
    us = 1e-6
    rccl = [30 * us, 40 * us, 80 * us, 400 * us, 1500 * us]
    inplace = [35 * us, 38 * us, 60 * us, 300 * us, 1100 * us]
    staged = [40 * us, 50 * us, 90 * us, 420 * us, 1700 * us]
    oneshot = [12 * us, 30 * us, 95 * us, inf, inf]
    p = decide(kb, rccl, inplace, staged, oneshot, world=8)
    # one-shot beats the in-place two-shot up to 1 MB, the staged one up to 1 MB as well
    assert p["oneshot_max_kb"] == 1024 and p["oneshot_max_staged_kb"] == 1024
    # registered path: 12 < 30, 30 < 40, 60 < 80, ... -> engine everywhere
    assert p["xgmi_min_kb_inplace"] == 0
    # staged: wins at 256 KB and 1 MB (one-shot) but loses from 4 MB on -> never
    assert p["xgmi_min_kb_staged"] is None
    # bandwidth knee: 128 MB is best (213 GB/s); 32 MB reaches 196 GB/s (> 85 %), 4 MB 122 GB/s
    bw = p["busbw_gbs"]
    assert bw[-1] == max(bw) and p["bucket_floor_mb"] == 32.0
    # a margin in RCCL's favour removes narrow wins (60 vs 80 us survives 10 %, 38 vs 40 does not)
    p = decide(kb, rccl, inplace, staged, [inf] * 5, world=8, margin=0.1)
    assert p["oneshot_max_kb"] == 0 and p["xgmi_min_kb_inplace"] == 4096


def test_median_table_ignores_inexact_and_mismatched_probes():
    from easydl_amd.parallel.comm_policy import median_table
    base = {"sizes_kb": [1024, 4096], "exact_everywhere": True, "xgmi_staged_ms": [1, 1], "xgmi_oneshot_ms": [1, None]}
    probes = [dict(base, sizes_kb=[1], rccl_ms=[5.0], xgmi_inplace_ms=[5.0]),     # older size grid: dropped
              dict(base, rccl_ms=[1.0, 2.0], xgmi_inplace_ms=[0.5, 9.0]),
              dict(base, rccl_ms=[3.0, 2.0], xgmi_inplace_ms=[0.7, 1.0]),
              dict(base, rccl_ms=[2.0, 2.0], xgmi_inplace_ms=[0.6, 1.0]),
              dict(base, rccl_ms=[99.0, 99.0], xgmi_inplace_ms=[0.1, 0.1], exact_everywhere=False)]
    t = median_table(probes)
    assert t is not None and t["n"] == 3 and t["sizes_kb"] == [1024, 4096]
    assert t["rccl_ms"] == [2.0, 2.0] and t["xgmi_inplace_ms"] == [0.6, 1.0]
    assert t["xgmi_oneshot_ms"][1] == float("inf")


def test_apply_allreduce_policy_routes_by_size():
    def fn(c, st):
        eng = FakeEngine(c, lambda nb: 0.0)
        eng.oneshot_max = eng.oneshot_max_staged = 0
        c.xgmi, c.xgmi_mode = eng, "xgmi"
        ok = c.apply_allreduce_policy({"xgmi_min_kb_inplace": 4096, "xgmi_min_kb_staged": None,
                                       "oneshot_max_kb": 512, "oneshot_max_staged_kb": 256})
        small = torch.zeros((1 << 20) // 4)         # 1 MB: RCCL
        big = torch.zeros((8 << 20) // 4)           # 8 MB: the engine (unregistered -> staged rule)
        return ok, c.xgmi_min_bytes, c.xgmi_min_bytes_staged, eng.oneshot_max, eng.oneshot_max_staged, \
            c._use_xgmi_allreduce(small), c._use_xgmi_allreduce(big)

    for ok, mi, ms, om, oms, u_small, u_big in _spawn(2, fn).values():
        assert ok and mi == 4 << 20 and ms == 1 << 62 and om == 512 << 10 and oms == 256 << 10
        assert not u_small and not u_big    # unregistered: staged rule says never


def test_probe_publishes_policy_with_oneshot_column():
    def fn(c, st):
        eng = FakeEngine(c, lambda nb: 0.0 if nb > (3 << 20) else 0.05)
        c.xgmi, c.xgmi_mode = eng, "auto"
        c._probe_xgmi(sizes_mb=(2, 4, 8), iters=1)
        return c.xgmi_probe, c.allreduce_policy

    for probe, pol in _spawn(2, fn).values():
        assert probe["sizes_kb"] == [2048, 4096, 8192]
        assert probe["xgmi_oneshot_ms"][2] is None and probe["xgmi_oneshot_ms"][0] is not None
        assert pol == probe["policy"] and pol["xgmi_min_kb_inplace"] == 4096


def test_probe_failure_on_one_rank_drops_the_engine_everywhere():
    """A form that raises on ONE rank mid-probe: every rank stops after that size (agreed
    over the control plane) and keeps RCCL only."""
    def fn(c, st):
        eng = FakeEngine(c, lambda nb: 0.0)
        real = eng.all_reduce

        def flaky(t, algo=None):
            if c.rank == 1 and eng.calls > 3 and algo == "twoshot":
                raise RuntimeError("launch failed")
            return real(t, algo)
        eng.all_reduce = flaky
        c.xgmi, c.xgmi_mode = eng, "auto"
        c._probe_xgmi(sizes_mb=(2, 4, 8), iters=1)
        return c.xgmi_probe, c.xgmi_mode, eng.closed

    for probe, mode, closed in _spawn(2, fn).values():
        assert probe["selected"] == "rccl" and mode is None and closed, probe


# --- policy cache and deferral (the recovery critical path measures nothing) -----------

def test_policy_cache_skips_the_probe_on_reformation():
    """Epoch 1 probes and caches the agreed table per (group, world); a later epoch of the
    same world adopts it in warmup without timing a single collective."""
    def fn(c, st):
        eng = FakeEngine(c, lambda nb: 0.0 if nb > (3 << 20) else 0.05)
        c.xgmi, c.xgmi_mode = eng, "auto"
        c.PROBE_KB = (2048, 4096, 8192)
        c._select_policy()
        first = dict(c.xgmi_probe)
        c.barrier()        # epochs are far apart in real life: the cache entry is written by now
        # the next epoch (a new communicator in real life): same group and world size
        eng2 = FakeEngine(c, lambda nb: 1.0)        # would flip the decision if it were timed
        c.xgmi, c.xgmi_mode, c.probe_mode, c.epoch = eng2, "auto", "defer", 2
        c._select_policy()
        return first, dict(c.xgmi_probe), eng2.calls, eng2.gate_calls, c.xgmi_mode, c.probe_pending

    for first, second, calls, gates, mode, pending in _spawn(2, fn).values():
        assert first["selected"] == "xgmi" and not first.get("cached")
        assert second["cached"] and second["measured_epoch"] == 1 and second["epoch"] == 2
        # no timing, but this epoch's engine passed the exactness gate (two-shot + one-shot)
        assert calls == 0 and gates == 2 and second["gate_exact"] is True
        assert mode == "xgmi" and not pending
        assert second["policy"] == first["policy"]


def test_cached_policy_is_refused_when_the_new_engine_is_not_exact():
    """A re-formed epoch whose engine mis-sums (e.g. a broken peer mapping) must not route
    gradients to it on the strength of an earlier epoch's cached verdict."""
    def fn(c, st):
        eng = FakeEngine(c, lambda nb: 0.0 if nb > (3 << 20) else 0.05)
        c.xgmi, c.xgmi_mode = eng, "auto"
        c.PROBE_KB = (2048, 4096, 8192)
        c._select_policy()
        c.barrier()
        eng2 = FakeEngine(c, lambda nb: 0.0, broken=c.rank == 1)   # only rank 1's sums are off
        c.xgmi, c.xgmi_mode, c.probe_mode, c.epoch = eng2, "auto", "defer", 2
        c._select_policy()
        return dict(c.xgmi_probe), c.xgmi_mode, eng2.closed

    for probe, mode, closed in _spawn(2, fn).values():
        assert probe["cached"] and probe["gate_exact"] is False
        assert probe["selected"] == "rccl" and mode is None and closed


def test_deferred_probe_runs_after_the_first_commit_only():
    """A re-formed epoch with no cached table routes everything to RCCL (no probe in
    warmup); run_deferred_probe() measures later, at an agreed point, and caches."""
    def fn(c, st):
        eng = FakeEngine(c, lambda nb: 0.0 if nb > (3 << 20) else 0.05)
        c.xgmi, c.xgmi_mode, c.probe_mode = eng, "auto", "defer"
        c.PROBE_KB = (2048, 4096, 8192)
        c._select_policy()
        before = (eng.calls, c.probe_pending, c._use_xgmi_allreduce(torch.zeros((8 << 20) // 4)))
        s = c.run_deferred_probe()
        key = c._policy_key()
        c.barrier()
        return before, s, eng.calls, c.xgmi_mode, c.probe_pending, st.check([key])

    for before, s, calls, mode, pending, cached in _spawn(2, fn).values():
        assert before == (0, True, False)            # nothing timed, RCCL carries every size
        assert s > 0 and calls > 0 and mode == "xgmi" and not pending and cached


def test_brain_policy_replaces_a_pending_probe():
    def fn(c, st):
        eng = FakeEngine(c, lambda nb: 0.2)
        c.xgmi, c.xgmi_mode, c.probe_mode = eng, "auto", "defer"
        c._select_policy()
        ok = c.adopt_policy({"xgmi_min_kb_inplace": 4096, "xgmi_min_kb_staged": 8192,
                             "oneshot_max_kb": 0, "oneshot_max_staged_kb": 0})
        return ok, eng.calls, c.xgmi_mode, c.probe_pending, c.xgmi_probe["source"], c.xgmi_min_bytes

    for ok, calls, mode, pending, src, mi in _spawn(2, fn).values():
        assert ok and calls == 0 and mode == "xgmi" and not pending and src == "brain" and mi == 4096 << 10


def test_policy_cache_needs_agreement():
    """A cache entry only some ranks can see (written between their reads) is ignored."""
    def fn(c, st):
        eng = FakeEngine(c, lambda nb: 0.0)
        c.xgmi, c.xgmi_mode = eng, "auto"
        if c.rank == 1:
            st.set(c._policy_key(), '{"exact_everywhere": true, "policy": {"xgmi_min_kb_inplace": 0}}')
        c.barrier()
        got = c._cached_policy()
        return got
    out = _spawn(2, fn)
    # both ranks read the same key after the barrier: agreed
    assert all(v is not None for v in out.values())


def test_rccl_p2p_batch_uses_the_coalescing_window_of_this_torch():
    """The multi-source state transfer on RCCL groups its sends and receives in
    ProcessGroupNCCL's coalescing window.  Pin the arity of that (private) API on the
    installed torch -- no argument, unlike older releases -- and drive _p2p_batch through
    a stand-in with exactly that interface (RCCL itself needs a rank per GPU)."""
    assert dist.ProcessGroupNCCL._start_coalescing.__doc__.startswith(
        "_start_coalescing(self: torch._C._distributed_c10d.Backend) -> None")
    assert dist.ProcessGroupNCCL._end_coalescing.__doc__.startswith(
        "_end_coalescing(self: torch._C._distributed_c10d.Backend) -> c10d::Work")
    calls = []

    class Work:
        def wait(self, *a):
            return True

        def is_completed(self):
            return True

    class FakeNCCL:
        def _start_coalescing(self):
            calls.append("start")

        def _end_coalescing(self):
            calls.append("end")
            return Work()

        def send(self, tensors, dst, tag):
            calls.append(("send", dst, tag))

        def recv(self, tensors, src, tag):
            calls.append(("recv", src, tag))

    c = Communicator.__new__(Communicator)
    c.data_kind, c.data = "rccl", FakeNCCL()
    c._wait = lambda w, poll=False: w.wait()
    t = torch.zeros(4)
    c._p2p_batch([("send", t, 1, 0), ("recv", t, 2, 0)])
    assert calls == ["start", ("send", 1, 0), ("recv", 2, 0), "end"]
