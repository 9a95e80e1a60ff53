"""In-memory snapshot through the native async D2H engine on the GPU + restore."""
import pytest
import torch

from easydl_amd.ckpt.manager import CheckpointManager, checksum_np, checksum_tensor, unlink_job_segments
from easydl_amd.models.llama import Llama, get_config
from easydl_amd.trainer.context import TrainerContext
from easydl_amd.trainer.data import SyntheticTokens
from easydl_amd.trainer.elastic import ElasticTrainer

pytestmark = pytest.mark.gpu
CFG = get_config("llama-tiny")


def _trainer(tmp, ckpt, seed, dev):
    ctx = TrainerContext(job="ckg", run_dir=str(tmp))
    return ElasticTrainer(lambda d: Llama(CFG, device=d), global_batch=2, micro_batch=2, lr=1e-3, device=dev,
                          ctx=ctx, checkpoint=ckpt, seed=seed)


def _flat(tr):
    return torch.cat([g.data.float() for g in tr.flat.groups] + [t.float() for t in tr.opt.state_tensors().values()])


def test_gpu_checksum_matches_reference(cuda):
    x = torch.randint(-2**31, 2**31 - 1, (1 << 20,), dtype=torch.int32, device=cuda)
    for n in (4, 1000, 4096, (1 << 20)):
        got = int(checksum_tensor(x[:n], base_index=7).item()) & ((1 << 64) - 1)
        assert got == checksum_np(x[:n].cpu().numpy().view("uint8"), 7)


def test_async_snapshot_and_restore(cuda, tmp_path):
    unlink_job_segments("ckg")
    data = SyntheticTokens(CFG.vocab_size, 64, num_samples=4096)
    ckpt = CheckpointManager("ckg", interval=2)
    try:
        a = _trainer(tmp_path, ckpt, 1, cuda)
        a.fit(lambda m, b: m(*b), data, num_steps=5)
        ckpt.wait()
        assert ckpt.last_snapshot_step == 4 and ckpt.stats["snapshots"] == 2
        a.fit  # keep alive
        b = _trainer(tmp_path, CheckpointManager("ckg", interval=1000), 2, cuda)
        b.fit(lambda m, b_: m(*b_), data, num_steps=4)   # restores step 4: nothing left to do
        assert b.step == 4
        ref = _trainer(tmp_path, None, 1, cuda)
        ref.fit(lambda m, b_: m(*b_), data, num_steps=4)
        assert torch.equal(_flat(b), _flat(ref))
    finally:
        ckpt.close()
        unlink_job_segments("ckg")


def test_restore_right_after_enqueue_drains_the_inflight_snapshot(cuda, tmp_path):
    """restore_latest() right after a snapshot was enqueued (the DP x TP rollback path):
    the in-flight D2H is drained first, so the slot it commits is consistent and a
    second restore of the same step still verifies."""
    unlink_job_segments("ckg")
    data = SyntheticTokens(CFG.vocab_size, 64, num_samples=4096)
    ckpt = CheckpointManager("ckg", interval=2)
    try:
        a = _trainer(tmp_path, ckpt, 1, cuda)
        a.fit(lambda m, b: m(*b), data, num_steps=4)     # snapshot of step 4 still in flight
        assert ckpt._ticket is not None
        expect = _flat(a).clone()
        assert ckpt.restore_latest(a) is not None and a.step == 4
        assert torch.equal(_flat(a), expect)
        a.fit(lambda m, b: m(*b), data, num_steps=6)     # step 6 enqueued ...
        assert ckpt.restore_latest(a, max_step=4) is not None and a.step == 4   # ... roll back to 4
        assert torch.equal(_flat(a), expect)
        assert ckpt.latest_step(a) == 6
    finally:
        ckpt.close()
        unlink_job_segments("ckg")


def test_lean_snapshot_through_the_d2h_engine(cuda, tmp_path):
    """Lean mode on the GPU path (native D2H engine + pipelined restore): the bf16 model
    is rebuilt from the restored fp32 master, the moments restart from zero."""
    unlink_job_segments("ckg")
    data = SyntheticTokens(CFG.vocab_size, 64, num_samples=4096)
    ckpt = CheckpointManager("ckg", interval=2, lean="always")
    try:
        a = _trainer(tmp_path, ckpt, 1, cuda)
        a.fit(lambda m, b: m(*b), data, num_steps=4)
        ckpt.wait()
        assert ckpt.mode == "lean" and ckpt.last_snapshot_step == 4
        master = {n: t.clone() for n, t in a.opt.state_tensors().items() if n.endswith(".master")}
        model = [g.data.clone() for g in a.flat.groups]
        b = _trainer(tmp_path, CheckpointManager("ckg", interval=1000), 2, cuda)
        b.fit(lambda m, b_: m(*b_), data, num_steps=4)   # restores step 4
        assert b.step == 4 and b.opt.moment_origin == 4
        st = b.opt.state_tensors()
        assert all(torch.equal(st[n], t) for n, t in master.items())
        assert all(torch.equal(g.data, w) for g, w in zip(b.flat.groups, model))
        assert all(float(st[n].abs().max()) == 0 for n in b.opt.moment_names())
    finally:
        ckpt.close()
        unlink_job_segments("ckg")


def test_staged_snapshots_into_an_adopted_segment_resume_bit_exactly(cuda, tmp_path, monkeypatch):
    """Pageable slots (EDL_SNAPSHOT_PIN=0 path): snapshots stream through a 2-deep ring of
    1 MiB pinned stages, so one snapshot wraps the ring many times.  A restarted trainer
    adopts the segment it restored from (no unmap, no page-locking) and keeps snapshotting
    into it; a third one restores the adopted segment's newest step and matches an
    uninterrupted run bit for bit."""
    monkeypatch.setenv("EDL_CKPT_STAGE_MB", "1")
    monkeypatch.setenv("EDL_CKPT_STAGES", "2")
    monkeypatch.setenv("EDL_CKPT_COPY_THREADS", "3")
    unlink_job_segments("ckg")
    data = SyntheticTokens(CFG.vocab_size, 64, num_samples=4096)
    ck_a, ck_b = CheckpointManager("ckg", interval=2, pin=False), CheckpointManager("ckg", interval=2, pin=False)
    try:
        a = _trainer(tmp_path, ck_a, 1, cuda)
        a.fit(lambda m, b: m(*b), data, num_steps=5)
        ck_a.wait()
        assert not ck_a._seg.pinned and ck_a.stats["staged_last"]["mb"] > 4
        b = _trainer(tmp_path, ck_b, 2, cuda)
        b.fit(lambda m, b_: m(*b_), data, num_steps=8)   # restores step 4, snapshots 6 and 8
        ck_b.wait()
        assert ck_b.stats.get("adopted") == 1 and not ck_b._seg.pinned
        # (a snapshot may be skipped while the adopted segment's pages are still being populated)
        assert ck_b.last_snapshot_step == 8
        assert ck_b.stats["snapshots"] + ck_b.stats.get("skipped_populating", 0) == 2
        c = _trainer(tmp_path, CheckpointManager("ckg", interval=1000), 3, cuda)
        c.fit(lambda m, b_: m(*b_), data, num_steps=8)   # restores step 8
        assert c.step == 8
        ref = _trainer(tmp_path, None, 1, cuda)
        ref.fit(lambda m, b_: m(*b_), data, num_steps=8)
        assert torch.equal(_flat(c), _flat(ref))
    finally:
        ck_a.close()
        ck_b.close()
        unlink_job_segments("ckg")


def test_restore_with_deferred_moments_is_bit_exact_and_verified(cuda, tmp_path):
    """World-1 restore (ElasticTrainer._sync_state): the master weights come back before the
    first step, the Adam moments on a side stream under it (CheckpointManager.restore_latest
    ``defer_moments``); the update waits for them and the whole checksum.  Training then matches
    an uninterrupted run bit for bit; a corrupted moment byte is caught before the update."""
    from easydl_amd.ckpt import manager as ckm
    unlink_job_segments("ckg")
    data = SyntheticTokens(CFG.vocab_size, 64, num_samples=4096)
    ckpt = CheckpointManager("ckg", interval=2)
    try:
        a = _trainer(tmp_path, ckpt, 1, cuda)
        a.fit(lambda m, b: m(*b), data, num_steps=5)
        ckpt.wait()
        assert ckpt.last_snapshot_step == 4
        ck_b = CheckpointManager("ckg", interval=1000)
        b = _trainer(tmp_path, ck_b, 2, cuda)
        b.fit(lambda m, b_: m(*b_), data, num_steps=7)       # restores step 4, moments deferred
        assert ckm.LAST_RESTORE_STATS.get("deferred_bytes", 0) > 0, ckm.LAST_RESTORE_STATS
        assert "deferred_restore_wait_s" in ck_b.stats and not ck_b._deferred
        ref = _trainer(tmp_path, None, 1, cuda)
        ref.fit(lambda m, b_: m(*b_), data, num_steps=7)
        assert torch.equal(_flat(b), _flat(ref))

        # a flipped byte inside a moment tensor of the newest slot: the deferred half fails the check
        from easydl_amd.ckpt.manager import ShmSegment
        tag = ck_b._tag(b)
        world, step, infos = ck_b.find_latest(tag)
        seg = ShmSegment(ck_b.seg_name(world, 0, tag), create=False)
        try:
            ent = next(e for e in infos[0]["meta"]["t"] if e[0].endswith(".m") and e[4] > e[3])
            v = seg.view(infos[0]["slot"], ent[5], 4)
            v[1] ^= 0x40
        finally:
            seg.close()
        c = _trainer(tmp_path, CheckpointManager("ckg", interval=1000), 3, cuda)
        with pytest.raises(RuntimeError, match="deferred moments"):
            c.fit(lambda m, b_: m(*b_), data, num_steps=9)   # raised at the first update's fence
    finally:
        ckpt.close()
        unlink_job_segments("ckg")
