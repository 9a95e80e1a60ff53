"""Checkpoint format v1 + shm A/B store + restore (CPU tier; GPU variant in test_ckpt_gpu)."""

import os

import numpy as np
import torch

from easydl_amd.ckpt.manager import CheckpointManager, ShmSegment, checksum_np, load_dir, shard_layout, \
    unlink_job_segments
from easydl_amd.models.llama import Llama, get_config
from easydl_amd.trainer.context import TrainerContext
from easydl_amd.trainer.data import SyntheticTokens
from easydl_amd.trainer.elastic import ElasticTrainer

# Per-process job name: under pytest-xdist the tests of this file run in several
# workers at once, and a shared name would let one test unlink another's shm slots.
JOB = f"ck{os.getpid()}"
CFG = get_config("llama-tiny", n_layers=1, dim=64, n_heads=4, n_kv_heads=2, ffn_dim=128, vocab_size=128)


def _trainer(tmp, ckpt, seed=1234):
    ctx = TrainerContext(job=JOB, run_dir=str(tmp))
    return ElasticTrainer(lambda d: Llama(CFG, device=d, dtype=torch.float32), global_batch=4, micro_batch=2,
                          lr=1e-3, device="cpu", ctx=ctx, checkpoint=ckpt, seed=seed)


def _flat(tr):
    return torch.cat([g.data.clone() for g in tr.flat.groups] + [t.clone() for t in tr.opt.state_tensors().values()])


def test_checksum_reference_properties():
    a = np.arange(1000, dtype=np.uint32).view(np.uint8)
    full = checksum_np(a)
    # piecewise with base index == whole
    assert (checksum_np(a[:400], 0) + checksum_np(a[400:], 100)) % (1 << 64) == full
    b = a.copy()
    b[4], b[8] = a[8], a[4]
    assert checksum_np(b) != full


def test_shard_layout_covers_everything():
    ts = [("a", torch.zeros(1001)), ("b", torch.zeros(7, dtype=torch.bfloat16))]
    seen = {"a": 0, "b": 0}
    for r in range(3):
        lay, end = shard_layout(ts, r, 3)
        for d in lay:
            seen[d["name"]] += d["hi"] - d["lo"]
            assert d["offset"] % 4096 == 0
    assert seen == {"a": 1001, "b": 7}


def test_shm_ab_slots_survive_torn_write():
    name = "/edl-test-ab-w1-s0"
    seg = ShmSegment(name, 1 << 20, create=True)
    try:
        s0 = seg.begin()
        seg.view(s0, 0, 4)[:] = [1, 2, 3, 4]
        seg.commit(s0, 10, 1, 4, 123, {"x": 1})
        s1 = seg.begin()
        assert s1 != s0
        seg.view(s1, 0, 4)[:] = [9, 9, 9, 9]  # torn: never committed
        again = ShmSegment(name, create=False)
        info = again.committed()
        assert [i["step"] for i in info] == [10] and info[0]["checksum"] == 123
        assert list(again.view(info[0]["slot"], 0, 4)) == [1, 2, 3, 4]
        again.close()
    finally:
        seg.close(unlink=True)


def test_snapshot_restore_resumes_bit_identically(tmp_path):
    unlink_job_segments(JOB)
    data = SyntheticTokens(CFG.vocab_size, 16, num_samples=1024)
    ref = _trainer(tmp_path, None)
    ref.fit(lambda m, b: m(*b), data, num_steps=10)
    ckpt = CheckpointManager(JOB, interval=3, persist_dir=str(tmp_path / "disk"), persist_every=1)
    try:
        a = _trainer(tmp_path, ckpt)
        a.fit(lambda m, b: m(*b), data, num_steps=7)
        ckpt.wait()
        assert ckpt.last_snapshot_step == 6
        # a brand-new process (different init) restores step 6 from /dev/shm and continues
        ckpt2 = CheckpointManager(JOB, interval=100)
        b = _trainer(tmp_path, ckpt2, seed=999)
        b.fit(lambda m, b_: m(*b_), data, num_steps=10)
        assert b.history[0]["step"] == 7  # resumed after step 6
        assert torch.equal(_flat(b), _flat(ref))
        # cold resume from disk (format v1)
        ckpt._persist_thread.join()
        c = _trainer(tmp_path, None, seed=5)
        load_dir(str(tmp_path / "disk" / "step-6"), c)
        assert c.step == 6
    finally:
        unlink_job_segments(JOB)


def test_restarted_trainer_adopts_the_segment_it_restored_from(tmp_path):
    """The restarted (only) worker keeps the mapping it restored from as its own snapshot
    segment: the next snapshot goes to the other A/B slot of that same mapping, and the
    restored step stays committed until the new one is."""
    unlink_job_segments(JOB)
    data = SyntheticTokens(CFG.vocab_size, 16, num_samples=1024)
    ckpt = CheckpointManager(JOB, interval=3)
    try:
        a = _trainer(tmp_path, ckpt)
        a.fit(lambda m, b: m(*b), data, num_steps=7)
        ckpt.wait()
        ckpt2 = CheckpointManager(JOB, interval=2)
        b = _trainer(tmp_path, ckpt2, seed=999)
        b.fit(lambda m, b_: m(*b_), data, num_steps=6)     # restore of step 6 only
        assert ckpt2.stats.get("adopted") == 1 and ckpt2._seg is not None
        seg = ckpt2._seg
        assert [i["step"] for i in seg.committed()] == [3, 6]
        b.fit(lambda m, b_: m(*b_), data, num_steps=8)     # snapshot of step 8 into the adopted mapping
        ckpt2.wait()
        assert ckpt2._seg is seg and sorted(i["step"] for i in seg.committed()) == [6, 8]
    finally:
        unlink_job_segments(JOB)


def test_snapshot_evaluator_reads_latest(tmp_path):
    from easydl_amd.trainer.evaluator import SnapshotEvaluator
    unlink_job_segments("ckev")
    data = SyntheticTokens(CFG.vocab_size, 16, num_samples=1024)
    ckpt = CheckpointManager("ckev", interval=2)
    try:
        ctx = TrainerContext(job="ckev", run_dir=str(tmp_path))
        tr = ElasticTrainer(lambda d: Llama(CFG, device=d, dtype=torch.float32), global_batch=4, micro_batch=2,
                            lr=1e-3, device="cpu", ctx=ctx, checkpoint=ckpt)
        tr.fit(lambda m, b: m(*b), data, num_steps=4)
        ev = SnapshotEvaluator(lambda d: Llama(CFG, device=d, dtype=torch.float32), "ckev", run_dir=str(tmp_path))
        res = ev.run(lambda m: {"loss": float(m(*data.batch([1, 2], "cpu")))}, interval_s=0, max_evals=1)
        assert res[0]["step"] == 4
        for a, b in zip(tr.flat.groups, ev.flat.groups):
            assert torch.equal(a.data, b.data)
    finally:
        unlink_job_segments("ckev")


def test_background_population_covers_every_slot():
    import time
    seg = ShmSegment("/edl-poptest-w1-s0", 48 << 20, create=True)
    try:
        assert seg.populated()                      # nothing started: nothing to wait for
        assert seg.populate_async(3) and not seg.populate_async(3)   # one population at a time
        t_end = time.time() + 30
        while not seg.populated() and time.time() < t_end:
            time.sleep(0.005)
        assert seg.populated()
        s0 = seg.begin()
        seg.view(s0, 0, 8)[:] = 5                   # the mapping stays usable
        assert int(seg.view(s0, 0, 8)[3]) == 5
    finally:
        seg.close(unlink=True)                      # joins the (finished) threads


def test_premapped_segments_are_reused_by_restore(tmp_path):
    """A hot standby maps + pre-faults the job's segments; the restore then uses that mapping."""
    from easydl_amd.ckpt import manager as m
    seg = m.ShmSegment("/edl-premaptest-w1-s0", 1 << 20, create=True)
    try:
        slot = seg.begin()
        seg.view(slot, 0, 16)[:] = 7
        seg.commit(slot, 3, 1, 16, 0, {})
        assert m.premap_job_segments("premaptest") == ["/edl-premaptest-w1-s0"]
        assert m.premap_job_segments("premaptest") == []              # already mapped
        s2 = m._open_segment("/edl-premaptest-w1-s0")
        assert s2.committed()[0]["step"] == 3 and int(s2.view(slot, 0, 16)[5]) == 7
        s2.close()
        assert "/edl-premaptest-w1-s0" not in m._PREMAPPED
    finally:
        seg.close(unlink=True)


def test_load_dir_latest_falls_back_past_a_torn_shard(tmp_path):
    """A corrupted newest step-* directory is skipped: cold resume uses the next older one."""
    unlink_job_segments(JOB)
    data = SyntheticTokens(CFG.vocab_size, 16, num_samples=1024)
    disk = tmp_path / "disk"
    ckpt = CheckpointManager(JOB, interval=2, persist_dir=str(disk), persist_every=1)
    try:
        a = _trainer(tmp_path, ckpt)
        a.fit(lambda m, b: m(*b), data, num_steps=6, on_step=lambda t, loss: ckpt._join_persist())
        ckpt.close()
        assert sorted(p.name for p in disk.iterdir()) == ["step-2", "step-4", "step-6"]
        shard = next((disk / "step-6").glob("*.bin"))
        raw = bytearray(shard.read_bytes())
        raw[100] ^= 0xFF
        shard.write_bytes(bytes(raw))
        unlink_job_segments(JOB)           # no in-memory copy left: the disk path is taken
        b = _trainer(tmp_path, None, seed=77)
        src = CheckpointManager(JOB, persist_dir=str(disk)).restore_latest(b)
        assert src == f"disk:{disk / 'step-4'}" and b.step == 4
    finally:
        unlink_job_segments(JOB)


def test_snapshot_skips_the_slot_a_persist_is_reading(tmp_path):
    """A/B slots: while the disk writer still reads slot X, the snapshot that would
    reuse X is skipped instead of tearing the file being written."""
    import threading
    unlink_job_segments(JOB)
    data = SyntheticTokens(CFG.vocab_size, 16, num_samples=1024)
    ckpt = CheckpointManager(JOB, interval=1)
    try:
        a = _trainer(tmp_path, ckpt)
        a.fit(lambda m, b: m(*b), data, num_steps=1)          # snapshot of step 1 -> slot s1
        release = threading.Event()
        ckpt._persist_thread = threading.Thread(target=release.wait, daemon=True)
        ckpt._persist_thread.start()
        ckpt._persist_slot = ckpt._last_slot                  # "persisting step 1"
        a.fit(lambda m, b: m(*b), data, num_steps=3)          # step 2 -> other slot; step 3 would reuse s1
        assert ckpt.stats.get("skipped", 0) == 1 and ckpt.last_snapshot_step == 2
        release.set()
        ckpt._join_persist()
        ckpt._persist_slot = None
        a.fit(lambda m, b: m(*b), data, num_steps=4)
        assert ckpt.last_snapshot_step == 4
    finally:
        ckpt.close()
        unlink_job_segments(JOB)


def test_world_change_reuses_the_pinned_segment(tmp_path):
    """A shrink by one rank re-uses the (headroom-sized, page-locked) segment under the
    new layout's name: no new mapping, no re-pinning.  The old layout's newest snapshot
    stays readable under the OLD name until this rank's first new-layout snapshot has
    committed (a whole-job restart in between still finds a complete world), and the
    new name never reports an old-layout slot as its own."""
    import os
    import types
    unlink_job_segments(JOB)
    ckpt = CheckpointManager(JOB, interval=1)
    try:
        a = _trainer(tmp_path, None)
        a.comm = types.SimpleNamespace(world_size=4, rank=1, epoch=1)
        a.step = 1
        ckpt.snapshot(a)
        ckpt.wait()
        h0 = ckpt._seg.h
        assert os.path.exists(f"/dev/shm/edl-{JOB}-w4-s1")
        a.comm = types.SimpleNamespace(world_size=3, rank=2, epoch=2)     # renumbered survivor
        a.step = 2
        seg = ckpt._segment(3, 2, shard_layout(CheckpointManager.state_of(a), 2, 3)[1] + 8)
        assert seg.h == h0 and ckpt.stats["reassigned"] == 1
        assert os.path.exists(f"/dev/shm/edl-{JOB}-w4-s1") and os.path.exists(f"/dev/shm/edl-{JOB}-w3-s2")
        old = ShmSegment(f"/edl-{JOB}-w4-s1", create=False)
        assert [i["step"] for i in old.committed()] == [1]                 # old world's snapshot kept
        old.close()
        assert [i["meta"]["world"] for i in seg.committed()] == [4]       # ... and tagged with its layout
        ckpt.snapshot(a)                                                   # first new-layout snapshot
        ckpt.wait()
        assert sorted(i["step"] for i in ckpt._seg.committed()) == [1, 2] and ckpt._seg.h == h0
        assert os.path.exists(f"/dev/shm/edl-{JOB}-w4-s1")
        a.step = 3
        ckpt.snapshot(a)                                                   # overwrites the kept slot
        ckpt.wait()
        assert not os.path.exists(f"/dev/shm/edl-{JOB}-w4-s1")
        assert sorted(i["step"] for i in ckpt._seg.committed()) == [2, 3]
    finally:
        ckpt.close()
        unlink_job_segments(JOB)


def test_find_latest_ignores_other_layout_slots(tmp_path):
    """A relinked segment shows old-layout slots under the new name: find_latest only
    counts slots whose recorded layout matches the name's (world, shard)."""
    import types
    unlink_job_segments(JOB)
    ckpt = CheckpointManager(JOB, interval=1)
    try:
        a = _trainer(tmp_path, None)
        a.comm = types.SimpleNamespace(world_size=1, rank=0, epoch=1)
        a.step = 5
        ckpt.snapshot(a)
        ckpt.wait()
        assert ckpt.find_latest()[:2] == (1, 5)
        # pretend the world-1 segment was relinked to a world-2 layout without a snapshot
        ckpt._seg.rt("edl_shm_relink", ckpt._seg.h, f"/edl-{JOB}-w2-s0".encode())
        seg1 = ShmSegment(f"/edl-{JOB}-w2-s1", slot_bytes=4096, create=True)
        seg1.commit(seg1.begin(), 5, 2, 8, 0, {"world": 2, "shard": 1, "t": []})
        found = ckpt.find_latest()
        assert found is not None and found[0] == 1     # not the half-matching world-2 set
        seg1.close()
    finally:
        ckpt.close()
        unlink_job_segments(JOB)


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


def test_module_buffers_are_training_state(tmp_path):
    """BatchNorm running statistics live in the flat buffer tensors that the snapshot,
    the persisted checkpoint and the joiner state broadcast carry."""
    unlink_job_segments("ckbn")

    def mk(ck, seed):
        ctx = TrainerContext(job="ckbn", run_dir=str(tmp_path))
        return ElasticTrainer(lambda d: _BNNet(d), global_batch=8, micro_batch=4, lr=1e-2, device="cpu", ctx=ctx,
                              checkpoint=ck, seed=seed)

    ckpt = CheckpointManager("ckbn", interval=3, persist_dir=str(tmp_path / "disk"), persist_every=1)
    try:
        a = mk(ckpt, 1)
        assert a.model.bn.running_mean.data_ptr() == a.bufs.tensors["float32"].data_ptr()
        a.fit(lambda m, b: m(*b), _Images(), num_steps=6)
        ckpt.wait()
        rm, rv, nb = (a.model.bn.running_mean.clone(), a.model.bn.running_var.clone(),
                      int(a.model.bn.num_batches_tracked))
        assert nb == 12 and not torch.allclose(rm, torch.zeros_like(rm))
        assert "model.buffers.float32" in dict(CheckpointManager.state_of(a))
        ckpt._persist_thread.join()
        c = mk(None, 7)
        load_dir(str(tmp_path / "disk" / "step-6"), c)
        assert torch.equal(c.model.bn.running_mean, rm) and torch.equal(c.model.bn.running_var, rv)
        assert int(c.model.bn.num_batches_tracked) == nb
    finally:
        unlink_job_segments("ckbn")


class _DropNet(torch.nn.Module):
    """Tiny token model with dropout: resume is only bit-exact if the random stream is."""

    def __init__(self, device=None):
        super().__init__()
        self.emb = torch.nn.Embedding(64, 32, device=device)
        self.fc1 = torch.nn.Linear(32, 64, device=device)
        self.drop = torch.nn.Dropout(0.3)
        self.fc2 = torch.nn.Linear(64, 64, device=device)

    def forward(self, ids, labels):
        h = self.drop(torch.relu(self.fc1(self.emb(ids))))
        return torch.nn.functional.cross_entropy(self.fc2(h).flatten(0, 1), labels.flatten())


def test_resume_is_bit_exact_with_dropout(tmp_path):
    """Snapshot at step 2 -> a NEW trainer (different constructor seed) restores it and
    trains to step 4: parameters and optimizer state equal an uninterrupted 4-step run
    bit for bit (per-step RNG streams + host state in the snapshot metadata)."""
    unlink_job_segments(JOB)
    data = SyntheticTokens(64, 16, num_samples=1024)

    def mk(ckpt, seed, sub):
        ctx = TrainerContext(job=JOB, run_dir=str(tmp_path / sub))
        return ElasticTrainer(lambda d: _DropNet(d), global_batch=4, micro_batch=2, lr=1e-2, device="cpu", ctx=ctx,
                              checkpoint=ckpt, seed=seed)

    ref = mk(None, 7, "a").fit(lambda m, b: m(*b), data, num_steps=4)
    ckpt = CheckpointManager(JOB, interval=2)
    try:
        mk(ckpt, 7, "b").fit(lambda m, b: m(*b), data, num_steps=2)
        ckpt.wait()
        resumed = mk(ckpt, 99, "c")     # wrong seed on purpose: the snapshot's host state wins
        resumed.fit(lambda m, b: m(*b), data, num_steps=4)
        assert resumed.step == 4 and resumed._seed == 7
        assert torch.equal(_flat(ref), _flat(resumed))
        info = ckpt.find_latest()
        assert info is not None and info[2][0]["meta"]["host"]["data"]["cursor_step"] == info[1]
    finally:
        ckpt.close()
        unlink_job_segments(JOB)


def test_host_budget_selects_lean_and_lean_restore_restarts_the_moments(tmp_path):
    """SURVEY.md §5.4 host-DRAM sizing: when two full slots do not fit the per-rank host
    budget but master-only slots do, snapshots go lean (no Adam moments); restoring one
    gives the weights back exactly, zeroes the moments and restarts the bias correction
    (moment_origin); with no room at all in-memory snapshots are off."""
    unlink_job_segments(JOB)
    data = SyntheticTokens(CFG.vocab_size, 16, num_samples=1024)
    sizing = _trainer(tmp_path, None)
    st = CheckpointManager.state_of(sizing)
    full = sum(t.numel() * t.element_size() for _, t in st)
    lean = sum(t.numel() * t.element_size() for n, t in st if not n.endswith((".m", ".v")))
    assert lean * 2 < full
    budget_gb = (2 * lean + 2 * full) / 2 / 2**30          # between two lean and two full slots
    ckpt = CheckpointManager(JOB, interval=2, host_budget_gb=budget_gb)
    try:
        a = _trainer(tmp_path, ckpt)
        a.fit(lambda m, b: m(*b), data, num_steps=4)
        ckpt.wait()
        assert ckpt.mode == "lean" and ckpt.stats["snapshots"] == 2
        info = max(ckpt._seg.committed(), key=lambda i: i["step"])
        assert info["meta"]["lean"] and not any(n.endswith((".m", ".v")) for n, *_ in info["meta"]["t"])
        weights = [g.data.clone() for g in a.flat.groups]
        with torch.no_grad():
            for g in a.flat.groups:
                g.data.add_(1.0)
            for t in a.opt.state_tensors().values():
                t.add_(1.0)
        a.step = 99
        assert ckpt.restore_latest(a) is not None
        assert a.step == 4 and all(torch.equal(g.data, w) for g, w in zip(a.flat.groups, weights))
        assert all(float(a.opt.state_tensors()[n].abs().max()) == 0 for n in a.opt.moment_names())
        assert a.opt.moment_origin == a.opt.step_count == 4
        a.fit(lambda m, b: m(*b), data, num_steps=6)           # trains on from the warm restart
        assert a.step == 6 and torch.isfinite(torch.as_tensor(a.last_loss))
    finally:
        ckpt.close(unlink=True)
    off = CheckpointManager(JOB + "x", interval=1, host_budget_gb=1e-9)
    try:
        b = _trainer(tmp_path, off)
        b.fit(lambda m, b_: m(*b_), data, num_steps=2)
        assert off.mode == "off" and off.stats["skipped_host"] == 2 and off._seg is None
    finally:
        off.close(unlink=True)


def test_snapshot_mode_is_agreed_over_the_group():
    """One rank short of host memory makes the whole DP group lean (mixed layouts could
    not be restored together)."""
    import datetime
    import socket
    import threading
    import types

    import torch.distributed as dist
    from easydl_amd.parallel.comm import Communicator

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = {}

    def run(r):
        st = dist.TCPStore("127.0.0.1", port, 2, r == 0, timeout=datetime.timedelta(seconds=30))
        c = Communicator(st, r, 2, 1, device=torch.device("cpu"), job="ckm")
        m = CheckpointManager(f"{JOB}-agree{r}", host_budget_gb=(10.0 if r == 0 else 2.5e-6))
        tr = types.SimpleNamespace(comm=c)
        out[r] = (m._decide_mode(tr, c, (2, r, ""), full_bytes=1 << 20, lean_bytes=1 << 10),
                  m._decide_mode(tr, c, (2, r, ""), full_bytes=1 << 20, lean_bytes=1 << 10))  # cached
        c.shutdown()

    ts = [threading.Thread(target=run, args=(r,)) for r in range(2)]
    [t.start() for t in ts]
    [t.join(60) for t in ts]
    assert out == {0: ("lean", "lean"), 1: ("lean", "lean")}, out


def test_snapshot_agreement_failure_skips_the_snapshot_and_aborts(tmp_path):
    """a peer dying inside the first snapshot of a new layout (the mode
    agreement is a collective) must not escape on_step: the snapshot is skipped and the
    communicator marked aborted, so fit() reconfigures instead of ending."""
    import types

    from easydl_amd.parallel.comm import CommAborted

    class DeadPeerComm:
        world_size, rank, epoch = 2, 0, 3
        aborted = False

        def ctrl_all_reduce(self, values, op=None):
            raise CommAborted("peer died during the snapshot-mode agreement")

        def abort(self):
            self.aborted = True

    unlink_job_segments(JOB)
    ckpt = CheckpointManager(JOB, interval=1)
    try:
        a = _trainer(tmp_path, None)
        a.comm = DeadPeerComm()
        a.step = 1
        ckpt.on_step(a)
        assert a.comm.aborted and ckpt.stats["skipped_comm"] == 1 and ckpt.stats["snapshots"] == 0
        # unsharded snapshots are rank 0's alone: no agreement, so no collective at all
        solo = CheckpointManager(JOB + "u", interval=1, sharded=False)
        a.comm = DeadPeerComm()
        assert solo.prepare_layout(a) == "full" and not a.comm.aborted
        a.comm = types.SimpleNamespace(world_size=2, rank=1, epoch=3)
        assert solo.prepare_layout(a) is None
        solo.close(unlink=True)
    finally:
        ckpt.close()
        unlink_job_segments(JOB)


def test_drop_old_name_spares_a_name_another_segment_took(tmp_path):
    """after a shard permutation another rank's relink can take this rank's old
    layout name for its own live segment; dropping the old name must then keep it."""
    import os
    unlink_job_segments(JOB)
    a, b = CheckpointManager(JOB, interval=1), CheckpointManager(JOB, interval=1)
    try:
        a._segment(4, 1, 4096)                    # A: w4-s1
        b._segment(4, 2, 4096)                    # B: w4-s2
        a._segment(3, 1, 4096)                    # A shrinks to w3-s1, keeps w4-s1 as its old name
        assert a._old_name == f"/edl-{JOB}-w4-s1"
        b._segment(4, 1, 4096)                    # B re-links to w4-s1 (the name A still holds)
        b_ino = os.stat(f"/dev/shm/edl-{JOB}-w4-s1").st_ino
        a._drop_old_name()                        # must not unlink B's live name
        assert os.path.exists(f"/dev/shm/edl-{JOB}-w4-s1")
        assert os.stat(f"/dev/shm/edl-{JOB}-w4-s1").st_ino == b_ino
    finally:
        a.close()
        b.close()
        unlink_job_segments(JOB)
