"""HBM resume / adopted-buffer semantics on the CPU tier (both findings).

A hot standby builds its flat buffers on the dead worker's memory (utils/vram.py ``take``
with ``keep=True``).  Two guarantees:

* the HBM resume is allowed only when EVERY state tensor -- weights, fp32 master, AdamW
  moments and the module buffers (BatchNorm running statistics) -- was adopted; otherwise the
  process restores a snapshot instead;
* when nothing overwrites the adopted buffers (no HBM resume, no snapshot, no state
  transfer), they are reset to this process's seeded init: the state equals a fresh start.

The buffers here are CPU tensors standing in for IPC-mapped HBM; the step-mark read is
patched to report a worker that died between two updates."""
import subprocess

import torch

from easydl_amd.ckpt.manager import CheckpointManager, unlink_job_segments
from easydl_amd.trainer.context import TrainerContext
from easydl_amd.trainer.elastic import ElasticTrainer
from easydl_amd.utils import stepmarks, vram


class _BNNet(torch.nn.Module):
    def __init__(self, device=None):
        super().__init__()
        self.conv = torch.nn.Conv2d(3, 8, 3, padding=1, device=device)
        self.bn = torch.nn.BatchNorm2d(8, device=device)
        self.fc = torch.nn.Linear(8, 5, device=device)

    def forward(self, x, y):
        h = torch.relu(self.bn(self.conv(x))).mean((2, 3))
        return torch.nn.functional.cross_entropy(self.fc(h), y)


class _Images:
    def __len__(self):
        return 4096

    def batch(self, idx, device="cpu"):
        idx = list(idx)
        g = torch.Generator().manual_seed(int(idx[0]))
        return torch.randn(len(idx), 3, 6, 6, generator=g) * 3 + 1, torch.tensor([i % 5 for i in idx])


JOB = "hbmres"


def _mk(tmp_path, seed, ckpt=None, sub="a"):
    ctx = TrainerContext(job=JOB, run_dir=str(tmp_path / sub))
    return ElasticTrainer(lambda d: _BNNet(d), global_batch=8, micro_batch=4, lr=1e-2, device="cpu", ctx=ctx,
                          checkpoint=ckpt, seed=seed)


def _state(t):
    out = {f"data.{g.name}": g.data.clone() for g in t.flat.groups}
    out.update({k: v.clone() for k, v in t.opt.state_tensors().items()})
    out.update({f"buf.{k}": v.clone() for k, v in t.bufs.tensors.items()})
    return out


def _dead_pid() -> int:
    p = subprocess.Popen(["true"])
    p.wait()
    return p.pid


def _died_worker(tmp_path, steps=3):
    """A worker trained ``steps`` steps; its buffers copied (the 'dead worker's HBM')."""
    a = _mk(tmp_path, 1, sub="dead")
    a.fit(lambda m, b: m(*b), _Images(), num_steps=steps)
    return a, {k: t.clone() for k, t in a.vram_state_tensors().items()}


def _marks(monkeypatch, k, pid):
    monkeypatch.setattr(stepmarks, "read_slot",
                        lambda job, slot, shadow=False: (k, k, pid) + ((0, 0, 0, 0) if shadow else ()))


def test_hbm_resume_adopts_every_state_tensor_including_batchnorm_buffers(tmp_path, monkeypatch):
    unlink_job_segments(JOB)
    dead, exported = _died_worker(tmp_path)
    assert {"bufs/float32", "bufs/int64"} <= set(exported)     # running stats + num_batches_tracked
    pid = _dead_pid()
    _marks(monkeypatch, 3, pid)
    vram.adopt(exported, pid=pid)
    ck = CheckpointManager(JOB, interval=100)
    try:
        b = _mk(tmp_path, 5, ck, sub="b")
        b.fit(lambda m, x: m(*x), _Images(), num_steps=3)   # resumes at 3: no step left to run
        ev = [r for r in b.events.records if r["kind"] in ("restored", "hbm_resume_refused", "adopted_reinit")]
        assert [r["kind"] for r in ev] == ["restored"] and ev[0]["source"] == "hbm:step3", ev
        assert b.step == 3
        got, want = _state(b), _state(dead)
        assert set(got) == set(want)
        for k in want:
            assert torch.equal(got[k], want[k]), k
        assert int(b.model.bn.num_batches_tracked) == int(dead.model.bn.num_batches_tracked) == 6
    finally:
        ck.close()
        unlink_job_segments(JOB)
        vram.adopt({})


def test_hbm_resume_refused_when_a_state_tensor_was_not_adopted(tmp_path, monkeypatch):
    """The running statistics were not exported: no HBM resume (it would pair the dead
    worker's weights with init statistics); no snapshot either, so a fresh seeded start."""
    unlink_job_segments(JOB)
    _, exported = _died_worker(tmp_path)
    del exported["bufs/float32"]
    pid = _dead_pid()
    _marks(monkeypatch, 3, pid)
    vram.adopt(exported, pid=pid)
    ck = CheckpointManager(JOB, interval=100)
    try:
        b = _mk(tmp_path, 5, ck, sub="b")
        b.fit(lambda m, x: m(*x), _Images(), num_steps=0)
        kinds = [r for r in b.events.records if r["kind"] in ("restored", "hbm_resume_refused", "adopted_reinit")]
        assert kinds[0]["kind"] == "hbm_resume_refused" and kinds[0]["reason"] == "incomplete"
        assert kinds[0]["missing"] == ["model.buffers.float32"]
        assert kinds[-1]["kind"] == "adopted_reinit" and b.step == 0
        vram.adopt({})
        fresh = _mk(tmp_path, 5, sub="c")
        got, want = _state(b), _state(fresh)
        for k in want:
            assert torch.equal(got[k], want[k]), k
        assert b.opt.step_count == 0 and b.opt.moment_origin == 0
    finally:
        ck.close()
        unlink_job_segments(JOB)
        vram.adopt({})


def test_adopted_buffers_without_resume_or_snapshot_equal_a_fresh_start(tmp_path, monkeypatch):
    """Marks refused (the worker died inside an update) and no checkpoint manager at all: the
    torn weights and non-zero moments must not survive into training."""
    _, exported = _died_worker(tmp_path)
    pid = _dead_pid()
    monkeypatch.setattr(stepmarks, "read_slot",
                        lambda job, slot, shadow=False: (4, 3, pid) + ((0,) * 4 if shadow else ()))   # begin != done
    vram.adopt(exported, pid=pid)
    try:
        b = _mk(tmp_path, 5, None, sub="b")
        assert vram.adopted_any()
        b.fit(lambda m, x: m(*x), _Images(), num_steps=0)
        vram.adopt({})
        fresh = _mk(tmp_path, 5, sub="c")
        got, want = _state(b), _state(fresh)
        for k in want:
            assert torch.equal(got[k], want[k]), k
        # and training from there matches the fresh process step for step
        b.fit(lambda m, x: m(*x), _Images(), num_steps=2)
        fresh.fit(lambda m, x: m(*x), _Images(), num_steps=2)
        got, want = _state(b), _state(fresh)
        for k in want:
            assert torch.equal(got[k], want[k]), k
    finally:
        vram.adopt({})


def test_unused_adopted_buffers_are_released(tmp_path):
    """Adopted tensors that no buffer asks for (here: the momentum buffer of an SGD worker,
    adopted by an AdamW process) are dropped right after the model is built, not kept mapped
    for the life of the process; a size / dtype mismatch is dropped at the ``take``."""
    _, exported = _died_worker(tmp_path)
    g = next(k for k in exported if k.endswith("/grad"))
    exported[g] = exported[g].double()
    exported["opt/decay/mom"] = torch.zeros(4)
    vram.adopt(exported, pid=_dead_pid())
    try:
        b = _mk(tmp_path, 5, None, sub="b")
        built = next(r for r in b.events.records if r["kind"] == "model_built")
        assert built["adopted_unused"] == 1
        assert not vram._ADOPTED
    finally:
        vram.adopt({})


def test_memory_limited_recovery_splits_micro_batches_with_the_same_update(tmp_path):
    """A replacement short of HBM (the dead worker's activations not reclaimed yet) runs each
    micro-batch as smaller ones: same samples, same weights -> the same update (up to the
    order of the additions).  The plan is re-made before every micro-batch, but inside a step it
    may only shrink (larger pieces need fresh allocator segments, slow right after the driver's
    reclaim): memory that comes back during the first step -- here between its first and second
    micro-batch -- gives full micro-batches from the next step on."""
    from easydl_amd.trainer.data import SyntheticTokens

    class _Tok(torch.nn.Module):
        def __init__(self, device=None):
            super().__init__()
            self.emb = torch.nn.Embedding(64, 32, device=device)
            self.fc = torch.nn.Linear(32, 64, device=device)

        def forward(self, ids, labels):
            return torch.nn.functional.cross_entropy(self.fc(torch.tanh(self.emb(ids))).flatten(0, 1),
                                                     labels.flatten())

    data = SyntheticTokens(64, 16, num_samples=512)

    def mk(sub):
        ctx = TrainerContext(job="split", run_dir=str(tmp_path / sub))
        return ElasticTrainer(lambda d: _Tok(d), global_batch=8, micro_batch=4, lr=1e-2, device="cpu", ctx=ctx,
                              seed=3)

    ref = mk("ref").fit(lambda m, b: m(*b), data, num_steps=2)
    sp = mk("split")
    avail = {"v": 600}                  # 1000 B needed per micro-batch of 4: two pieces of 2 fit
    sp._hbm_avail = lambda: avail["v"]
    sp._act_need = 1000
    sp._mb_limited = True
    sp._memory_plan = lambda: None      # (on a GPU takeover: free HBM < the published need)
    orig = sp._replan_memory
    sizes = []

    def replan(mb, grow=True):
        orig(mb, grow)
        avail["v"] = 10_000             # the driver reclaims the memory during micro-batch 0
    sp._replan_memory = replan

    def loss_fn(m, b):
        sizes.append(int(b[0].shape[0]))
        return m(*b)
    sp.fit(loss_fn, data, num_steps=2)
    assert sizes == [2, 2, 2, 2, 4, 4], sizes
    kinds = [(r["kind"], r.get("mb")) for r in sp.events.records if r["kind"].startswith("memory_")]
    assert kinds == [("memory_replanned", 0), ("memory_restored", 0)], kinds
    for a, b in zip(ref.flat.groups, sp.flat.groups):
        assert torch.allclose(a.data, b.data, atol=1e-6, rtol=1e-5)


def test_resumed_state_is_rehomed_and_training_continues_bit_exactly(tmp_path, monkeypatch):
    """After an HBM resume the replacement moves the adopted buffers into its own memory at the
    first step boundary (ElasticTrainer._maybe_rehome: imported memory cannot be exported to the
    next standby) and trains on exactly as an uninterrupted run."""
    unlink_job_segments(JOB)
    monkeypatch.setenv("EDL_VRAM_HANDOFF", "1")
    _, exported = _died_worker(tmp_path)
    pid = _dead_pid()
    _marks(monkeypatch, 3, pid)
    vram.adopt(exported, pid=pid)
    ck = CheckpointManager(JOB, interval=100)
    try:
        b = _mk(tmp_path, 5, ck, sub="b")
        b.fit(lambda m, x: m(*x), _Images(), num_steps=6)
        kinds = [r["kind"] for r in b.events.records]
        assert "rehomed" in kinds and kinds.count("rehomed") == 1, kinds
        ev = next(r for r in b.events.records if r["kind"] == "rehomed")
        assert ev["step"] == 4 and ev["buffers"] == len(exported), ev
        adopted_ptrs = {t.data_ptr() for t in exported.values()}
        mine = b.vram_state_tensors()
        assert not ({t.data_ptr() for t in mine.values()} & adopted_ptrs)   # nothing left on adopted memory
        for g in b.flat.groups:                                             # params view the new buffers
            for s in g.slots:
                assert s.param.data_ptr() == g.data[s.offset:].data_ptr()
        assert not vram.adopted_any()      # (on a GPU it is re-published for the next standby here)
        ref = _mk(tmp_path, 1, sub="ref")
        ref.fit(lambda m, x: m(*x), _Images(), num_steps=6)
        got, want = _state(b), _state(ref)
        for k in want:
            assert torch.equal(got[k], want[k]), k
    finally:
        ck.close()
        unlink_job_segments(JOB)
        vram.adopt({})


def test_mid_step_resume_from_the_gradient_shadow_is_bit_exact(tmp_path, monkeypatch):
    """The worker dies in step 4 after 2 of its 4 micro-batches (the gradient buffer itself is
    torn: a backward was in flight).  Its shadow holds the gradients of micro-batches 0-1 and
    the partial loss, its step marks say (gstep, gmb) = (4, 2): the replacement resumes step 4
    at micro-batch 2 and ends bit-identical to an uninterrupted run -- BatchNorm running
    statistics included, which a whole-step replay would have updated twice."""
    unlink_job_segments(JOB)
    pid = _dead_pid()

    def mk(sub, seed, ckpt=None):
        ctx = TrainerContext(job=JOB, run_dir=str(tmp_path / sub))
        return ElasticTrainer(lambda d: _BNNet(d), global_batch=16, micro_batch=4, lr=1e-2, device="cpu",
                              ctx=ctx, checkpoint=ckpt, seed=seed)

    a = mk("dead", 1)
    a.fit(lambda m, b: m(*b), _Images(), num_steps=3)
    a._marks = stepmarks.StepMarks(JOB, "shadowtest")      # host-written page (CPU)
    a.flat.ensure_shadow()
    calls = {"n": 0}

    def dies(m, b):
        calls["n"] += 1
        if calls["n"] == 3:
            raise KeyboardInterrupt("killed before micro-batch 2 of step 4")
        return m(*b)
    try:
        a.fit(dies, _Images(), num_steps=4)
    except KeyboardInterrupt:
        pass
    assert a.step == 3 and a._marks.read_shadow() == (4, 2)
    for g in a.flat.groups:
        g.grad.add_(1.0)            # the in-flight backward's partial adds: the shadow must be used
    exported = {k: t.clone() for k, t in a.vram_state_tensors().items()}
    a._marks.close(unlink=True)
    assert "flat/gshadow_loss" in exported
    monkeypatch.setattr(stepmarks, "read_slot",
                        lambda job, slot, shadow=False: (3, 3, pid) + ((4, 2, 0, 0) if shadow else ()))
    vram.adopt(exported, pid=pid)
    ck = CheckpointManager(JOB, interval=100)
    try:
        b = mk("b", 5, ck)
        b.fit(lambda m, x: m(*x), _Images(), num_steps=6)
        ev = [r for r in b.events.records if r["kind"] in ("restored", "resumed_mid_step")]
        assert [r["kind"] for r in ev] == ["restored", "resumed_mid_step"], ev
        assert ev[1]["step"] == 4 and ev[1]["micro_batches_done"] == 2 and ev[1]["of"] == 4
        vram.adopt({})
        ref = mk("ref", 1).fit(lambda m, x: m(*x), _Images(), num_steps=6)
        got, want = _state(b), _state(ref)
        for k in want:
            assert torch.equal(got[k], want[k]), k
        assert int(b.model.bn.num_batches_tracked) == int(ref.model.bn.num_batches_tracked) == 24
    finally:
        ck.close()
        unlink_job_segments(JOB)
        vram.adopt({})


def test_no_rehome_while_other_ranks_train(tmp_path):
    """Re-homing is one rank's move, and re-registering its gradient buffers with the xGMI engine
    would be collective: a replacement in a world of several ranks keeps the adopted buffers (a
    world-8 drill hung there).  The move happens once the world is one rank."""
    from types import SimpleNamespace
    _, exported = _died_worker(tmp_path)
    vram.adopt(exported, pid=_dead_pid())
    try:
        b = _mk(tmp_path, 5, None, sub="b")
        assert vram.adopted_any()
        b.comm = SimpleNamespace(world_size=8)
        b._maybe_rehome()
        assert vram.adopted_any() and not b._rehomed
        assert "rehomed" not in [r["kind"] for r in b.events.records]
        b.comm = SimpleNamespace(world_size=1)
        b._maybe_rehome()
        assert b._rehomed and not vram.adopted_any()
    finally:
        vram.adopt({})
