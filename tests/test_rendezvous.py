"""RendezvousManager state machine (easydl_amd/master/rendezvous.py) driven tick by
tick on an in-memory store with a fake clock: epoch formation, join window,
scale-up admission of joiners that are still warming up, failure shrink,
replace policy and TP-aware re-ranking."""
import json

import torch.distributed as dist

from easydl_amd.master.rendezvous import RendezvousConfig, RendezvousManager
from easydl_amd.master.store import KV


class Clock:
    def __init__(self):
        self.t = 1000.0

    def __call__(self):
        return self.t


def _setup(**cfg):
    kv = KV(dist.HashStore(), "edl/t")
    clk = Clock()
    m = RendezvousManager(kv, RendezvousConfig(**cfg), clock=clk)
    return kv, clk, m


def _join(kv, clk, node):
    kv.set(f"hb/{node}", str(clk.t))
    kv.append("rdzv/joined", node + ",")


def _arrive(kv, clk, node):
    kv.set(f"rdzv/arrive_ts/{node}", str(clk.t))
    kv.append("rdzv/arriving", node + ",")


def _assign(kv, e):
    return json.loads(kv.get_str(f"rdzv/assign/{e}"))


def _beat(kv, clk, *nodes):
    for n in nodes:
        kv.set(f"hb/{n}", str(clk.t))


def _form_first(m, clk, kv, *nodes):
    """Initial epoch: the first tick opens the join window (or forms at once when
    max_nodes are present), a tick after the window forms."""
    e = m.tick()
    if e is not None:
        return e
    clk.t += m.cfg.join_window_s + 0.05
    _beat(kv, clk, *nodes)
    return m.tick()


def test_initial_epoch_waits_for_the_join_window():
    kv, clk, m = _setup(min_nodes=1, max_nodes=4, join_window_s=0.5)
    _join(kv, clk, "a")
    assert m.tick() is None                      # window starts
    clk.t += 0.2
    _join(kv, clk, "b")
    assert m.tick() is None
    clk.t += 0.4
    assert m.tick() == 1
    a = _assign(kv, 1)
    assert a["members"] == ["a", "b"] and a["reason"] == "initial"


def test_scale_up_joins_after_window_or_at_target():
    kv, clk, m = _setup(min_nodes=1, max_nodes=3, join_window_s=0.5)
    _join(kv, clk, "a")
    assert _form_first(m, clk, kv, "a") == 1
    _join(kv, clk, "b")
    _beat(kv, clk, "a")
    assert m.tick() is None                      # below target: wait for the window
    clk.t += 0.6
    _beat(kv, clk, "a", "b")
    assert m.tick() == 2 and _assign(kv, 2)["members"] == ["a", "b"]
    _join(kv, clk, "c")
    assert m.tick() == 3 and _assign(kv, 3)["world"] == 3   # target reached: no window


def test_scale_up_waits_for_joiners_still_warming_up():
    """Two joiners of one scale event: the second is still in its pre-join warm-up when
    the window ends.  The master holds the epoch for it: one re-formation, not two."""
    kv, clk, m = _setup(min_nodes=1, max_nodes=4, join_window_s=0.5, arrive_timeout_s=30)
    _join(kv, clk, "a")
    assert _form_first(m, clk, kv, "a") == 1
    _arrive(kv, clk, "b")
    _arrive(kv, clk, "c")
    clk.t += 1.0
    _join(kv, clk, "b")                          # b warmed up first
    _beat(kv, clk, "a")
    assert m.tick() is None
    clk.t += 2.0                                 # window long over, c still warming up
    _beat(kv, clk, "a", "b")
    assert m.tick() is None
    _join(kv, clk, "c")
    clk.t += 0.6
    _beat(kv, clk, "a", "b", "c")
    assert m.tick() == 2
    assert _assign(kv, 2)["members"] == ["a", "b", "c"]


def test_arrival_hold_expires():
    kv, clk, m = _setup(min_nodes=1, max_nodes=4, join_window_s=0.5, arrive_timeout_s=5)
    _join(kv, clk, "a")
    assert _form_first(m, clk, kv, "a") == 1
    _arrive(kv, clk, "b")
    _arrive(kv, clk, "c")                        # c never finishes its warm-up
    _join(kv, clk, "b")
    clk.t += 1.0
    _beat(kv, clk, "a", "b")
    assert m.tick() is None
    clk.t += 5.0
    _beat(kv, clk, "a", "b")
    assert m.tick() == 2 and _assign(kv, 2)["members"] == ["a", "b"]


def test_arrival_that_exits_releases_the_hold():
    kv, clk, m = _setup(min_nodes=1, max_nodes=4, join_window_s=0.5, arrive_timeout_s=30)
    _join(kv, clk, "a")
    assert _form_first(m, clk, kv, "a") == 1
    _arrive(kv, clk, "b")
    _arrive(kv, clk, "c")
    _join(kv, clk, "b")
    clk.t += 1.0
    _beat(kv, clk, "a", "b")
    assert m.tick() is None                      # c still starting
    kv.set("ev/exit/c", json.dumps({"code": 1}))  # ... and its process died before joining
    clk.t += 0.6                                 # past the join window: no arrival holds it now
    _beat(kv, clk, "a", "b")
    assert m.tick() == 2 and _assign(kv, 2)["members"] == ["a", "b"]


def test_failure_shrinks_and_aborts_the_broken_epoch():
    kv, clk, m = _setup(min_nodes=1, max_nodes=4, join_window_s=0.1)
    for n in "abc":
        _join(kv, clk, n)
    assert _form_first(m, clk, kv, *"abc") == 1
    kv.set("ev/dead/b", "process exit")
    assert m.tick() == 2
    assert kv.exists("rdzv/abort/1")
    a = _assign(kv, 2)
    assert a["members"] == ["a", "c"] and a["reason"] == "failure"


def test_heartbeat_timeout_marks_dead():
    kv, clk, m = _setup(min_nodes=1, max_nodes=4, join_window_s=0.1, heartbeat_timeout_s=3)
    for n in "ab":
        _join(kv, clk, n)
    assert _form_first(m, clk, kv, *"ab") == 1
    clk.t += 4
    _beat(kv, clk, "a")
    assert m.tick() == 2
    assert kv.exists("ev/dead/b") and _assign(kv, 2)["members"] == ["a"]


def test_replace_policy_waits_for_a_replacement():
    kv, clk, m = _setup(min_nodes=1, max_nodes=4, join_window_s=0.1, policy="replace", replace_wait_s=10)
    for n in "ab":
        _join(kv, clk, n)
    assert _form_first(m, clk, kv, *"ab") == 1
    kv.set("ev/dead/b", "process exit")
    assert m.tick() is None                      # waits for a replacement ...
    clk.t += 1
    _join(kv, clk, "b2")
    _beat(kv, clk, "a")
    assert m.tick() == 2 and _assign(kv, 2)["members"] == ["a", "b2"]


def test_tp_granule_keeps_survivor_tp_ranks():
    """granule 2 (TP=2): worlds are multiples of 2 and a survivor keeps rank % 2."""
    kv, clk, m = _setup(min_nodes=2, max_nodes=4, join_window_s=0.1, granule=2)
    for n in "abcd":
        _join(kv, clk, n)
    assert _form_first(m, clk, kv, *"abcd") == 1
    kv.set("ev/dead/a", "process exit")          # a had rank 0 (TP rank 0)
    assert m.tick() == 2
    a2 = _assign(kv, 2)
    assert a2["world"] == 2                      # 3 survivors -> one TP pair
    for node in a2["members"]:
        assert a2["members"].index(node) % 2 == ["a", "b", "c", "d"].index(node) % 2
