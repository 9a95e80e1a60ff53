"""Fault-injection specs (utils/fault.py): parsing and where each point fires.

The drills measure recovery from these faults, so a spec that fires at the wrong place (or not
at all) silently changes what a time-to-recover number means."""
from easydl_amd.utils.fault import FaultInjector, FaultSpec


class _Recorder(FaultInjector):
    def __init__(self, specs, **kw):
        super().__init__(specs, **kw)
        self.fired = []

    def _fire(self, s, trainer):
        self.fired.append((s.kind, s.point, s.mb))


def test_parse_microbatch_point():
    (s,) = FaultSpec.parse("kill@step=4,index=0,point=microbatch,mb=3,wait=standby")
    assert (s.kind, s.step, s.index, s.point, s.mb, s.wait) == ("kill", 4, 0, "microbatch", 3, "standby")
    (t,) = FaultSpec.parse("kill@step=2")
    assert t.point == "step_start" and t.mb == -1 and t.after_ms == 0


def test_microbatch_point_fires_only_after_its_micro_batch():
    inj = _Recorder(FaultSpec.parse("kill@step=4,point=microbatch,mb=2"), index=0)
    for step in (3, 4):
        inj.maybe_inject("step_start", step)
        for mb in range(4):
            inj.maybe_inject("microbatch", step, mb=mb)
    assert inj.fired == [("kill", "microbatch", 2)]


def test_index_role_and_generation_filters():
    specs = FaultSpec.parse("kill@step=1,index=1;exit@step=1,role=ps;raise@step=1,gen=1")
    inj = _Recorder(specs, index=0, role="worker", generation=0)
    inj.maybe_inject("step_start", 1)
    assert inj.fired == []
    inj2 = _Recorder(FaultSpec.parse("kill@step=1,index=1;exit@step=1,role=ps;raise@step=1,gen=1"),
                     index=1, role="ps", generation=0)
    inj2.maybe_inject("step_start", 1)
    assert [k for k, _, _ in inj2.fired] == ["kill", "exit"]       # a replacement (gen 1) only fires gen=1
    inj3 = _Recorder(FaultSpec.parse("kill@step=1;raise@step=1,gen=1"), generation=1)
    inj3.maybe_inject("step_start", 1)
    assert [k for k, _, _ in inj3.fired] == ["raise"]


def test_best_shadow_picks_the_fullest_valid_slot_of_the_step():
    from easydl_amd.utils.stepmarks import best_shadow
    assert best_shadow((5, 1, 5, 2), 5) == (1, 2)
    assert best_shadow((5, 3, 5, 0), 5) == (0, 3)        # slot 1 invalidated mid-copy
    assert best_shadow((5, 1, 4, 3), 5) == (0, 1)        # slot 1 is the previous step's
    assert best_shadow((4, 3, 4, 2), 5) is None
    assert best_shadow((5, 0, 5, 0), 5) is None
    assert best_shadow((5, 2), 5) == (0, 2)              # the HBM shadow: one slot
