"""VRAM hand-over from a dead worker to the hot standby (easydl_amd/utils/vram.py).

CPU tier: the allocation side (FlatParams / FlatAdamW build on adopted buffers, the group cap,
mismatches fall back to allocation).  GPU tier: a real IPC export by a child process, imported
here, still readable after the child has exited, and adopted by the next FlatParams/FlatAdamW.
"""
import os
import subprocess
import sys
import time

import pytest
import torch

from easydl_amd.optim import FlatAdamW
from easydl_amd.parallel.flat import FlatParams
from easydl_amd.utils import vram

HERE = os.path.dirname(os.path.abspath(__file__))


def _model(seed, device="cpu"):
    torch.manual_seed(seed)
    return torch.nn.Sequential(torch.nn.Linear(64, 128), torch.nn.ReLU(), torch.nn.Linear(128, 32)).to(device)


def _state(flat, opt):
    ts = {}
    for g in flat.groups:
        ts[f"flat/{g.name}/data"], ts[f"flat/{g.name}/grad"] = g.data, g.grad
    for g, st in zip(flat.groups, opt.state):
        for k, t in st.items():
            if isinstance(t, torch.Tensor) and t is not g.data:
                ts[f"opt/{g.name}/{k}"] = t
    return ts


def test_group_cap_under_handoff(monkeypatch):
    monkeypatch.setenv("EDL_VRAM_HANDOFF", "1")
    monkeypatch.delenv("EDL_FLAT_GROUP_MAX_MB", raising=False)
    assert vram.enabled() and vram.GROUP_MAX_MB * 2 * 2**20 < vram.IPC_MAX_BYTES
    # a 1,100 MiB-equivalent budget split: the cap bounds every group (fp32 state < 2 GiB)
    m = torch.nn.Sequential(*[torch.nn.Linear(64, 64, bias=False) for _ in range(4)]).to(torch.bfloat16)
    f = FlatParams(m, max_group_bytes=2 * 64 * 64 * 2)   # explicit cap still honoured
    assert len(f.groups) == 2


def test_flat_and_adamw_build_on_adopted_buffers():
    src = _model(1)
    f0 = FlatParams(src)
    o0 = FlatAdamW(f0)
    old = {k: t.clone().fill_(7.0) for k, t in _state(f0, o0).items()}
    vram.adopt(old)
    try:
        m = _model(2)
        f1 = FlatParams(m)
        o1 = FlatAdamW(f1)
        got = _state(f1, o1)
        assert set(got) == set(old)
        for k, t in got.items():
            assert t.data_ptr() == old[k].data_ptr(), k            # the adopted storage, not a copy
        for g, st in zip(f1.groups, o1.state):
            assert torch.count_nonzero(g.grad) == 0                   # gradients start from zero
            # the training state keeps the previous worker's values (an HBM resume needs them;
            # a restore / state transfer overwrites them otherwise)
            for t in (g.data, st["master"], st["m"], st["v"]):
                assert bool((t == 7.0).all())
        for p_new in m.parameters():                                   # the model now views that state
            assert bool((p_new.data == 7.0).all())
        assert vram.STATS["adopted"] >= len(old)
    finally:
        vram.release_unused()


def test_mismatched_buffer_is_not_adopted():
    vram.adopt({"flat/decay/data": torch.zeros(3)})
    try:
        f = FlatParams(_model(3))
        assert f.groups[0].data.numel() != 3
    finally:
        vram.release_unused()


def test_dead_pid():
    p = subprocess.Popen([sys.executable, "-c", "pass"])
    p.wait()
    assert vram.dead(p.pid) and not vram.dead(os.getpid())


@pytest.mark.gpu
def test_ipc_export_survives_the_exporter_and_is_adopted(cuda):
    import torch.distributed as dist

    from easydl_amd.master.store import KV
    store = dist.TCPStore("127.0.0.1", 0, is_master=True, wait_for_workers=False)
    kv = KV(store, "edl/vramtest")
    env = dict(os.environ, EDL_VRAM_HANDOFF="1", VT_PORT=str(store.port))
    child = subprocess.Popen([sys.executable, os.path.join(HERE, "helpers", "vram_export_proc.py")], env=env)
    try:
        assert kv.wait_for("vt/published", 120)
        held = vram.import_published(kv, "worker0")
        assert held and held["pid"] == child.pid and held["tensors"]
        kv.set("vt/imported", "1")
        assert child.wait(60) == 0
        t_end = time.time() + 10
        while not vram.dead(child.pid) and time.time() < t_end:
            time.sleep(0.05)
        # the exporter is gone; the imported memory still holds what it wrote
        for name, t in held["tensors"].items():
            assert float(t.float().mean()) == pytest.approx(3.0), name
        vram.adopt(held["tensors"])
        torch.manual_seed(5)
        m = torch.nn.Sequential(torch.nn.Linear(256, 512), torch.nn.Linear(512, 256)).to(cuda, torch.bfloat16)
        f = FlatParams(m)
        o = FlatAdamW(f)
        got = _state(f, o)
        assert all(got[k].data_ptr() == t.data_ptr() for k, t in held["tensors"].items())
        g = f.groups[0]
        g.grad.fill_(1)
        o.step()                                       # the adopted buffers are live device memory
        torch.cuda.synchronize()
        assert torch.isfinite(g.data.float()).all()
    finally:
        vram.release_unused()
        if child.poll() is None:
            child.kill()


def test_mm_released_tracks_a_killed_process():
    import signal as _signal

    from easydl_amd.utils.procfs import exit_status, mm_released
    assert not mm_released(os.getpid())
    p = subprocess.Popen([sys.executable, "-c", "import time; time.sleep(60)"])
    try:
        time.sleep(0.2)
        assert not mm_released(p.pid)
        os.kill(p.pid, _signal.SIGKILL)
        t_end = time.time() + 10
        while not mm_released(p.pid) and time.time() < t_end:   # a zombie holds no address space
            time.sleep(0.01)
        assert mm_released(p.pid) and vram.dead(p.pid)
        assert not vram.reaped(p.pid)                            # a zombie is not reaped yet
        assert exit_status(p.pid) == _signal.SIGKILL
    finally:
        p.wait()
    assert mm_released(p.pid) and vram.reaped(p.pid)


def test_exit_status_of_a_normal_exit_is_zero():
    from easydl_amd.utils.procfs import exit_status
    p = subprocess.Popen([sys.executable, "-c", "pass"])
    t_end = time.time() + 20
    while exit_status(p.pid) is not None and time.time() < t_end:
        st = exit_status(p.pid)
        with open(f"/proc/{p.pid}/stat") as f:
            zombie = f.read().rsplit(")", 1)[1].split()[0] == "Z"
        if zombie:
            assert st == 0          # exit(0): the operator waits for the reap (no early hand-over)
            break
        time.sleep(0.01)
    p.wait()


def test_step_marks_host_path(tmp_path):
    from easydl_amd.utils import stepmarks
    job = f"sm{os.getpid()}"
    m = stepmarks.StepMarks(job, "worker0")
    try:
        m.set_now(5)
        assert m.read() == (5, 5, os.getpid())
        m.begin(6)
        assert stepmarks.read_slot(job, "worker0")[:2] == (6, 5)      # an update in flight
        m.done(6)
        assert stepmarks.read_slot(job, "worker0")[:2] == (6, 6)
        assert stepmarks.read_slot(job, "worker9") is None
    finally:
        m.close(unlink=True)


def test_hbm_resume_continues_bit_exactly_without_a_restore(tmp_path):
    """A replacement that adopted a dead worker's state whose step marks say begin == done == 7
    resumes at step 7 from that state (no snapshot restored: the newest snapshot is step 6) and
    matches an uninterrupted run."""
    from easydl_amd.ckpt.manager import CheckpointManager, unlink_job_segments
    from easydl_amd.models.llama import Llama, get_config
    from easydl_amd.trainer.context import TrainerContext
    from easydl_amd.trainer.data import SyntheticTokens
    from easydl_amd.trainer.elastic import ElasticTrainer
    from easydl_amd.utils import stepmarks
    job = f"hbm{os.getpid()}"
    cfg = get_config("llama-tiny", n_layers=1, dim=64, n_heads=4, n_kv_heads=2, ffn_dim=128, vocab_size=128)
    data = SyntheticTokens(cfg.vocab_size, 16, num_samples=1024)

    def mk(ckpt, seed):
        ctx = TrainerContext(job=job, run_dir=str(tmp_path))
        return ElasticTrainer(lambda d: Llama(cfg, device=d, dtype=torch.float32), global_batch=4, micro_batch=2,
                              lr=1e-3, device="cpu", ctx=ctx, checkpoint=ckpt, seed=seed)

    unlink_job_segments(job)
    try:
        ref = mk(None, 1234)
        ref.fit(lambda m, b: m(*b), data, num_steps=10)
        a = mk(CheckpointManager(job, interval=3), 1234)
        a.fit(lambda m, b: m(*b), data, num_steps=7)       # snapshots of 3 and 6; HBM at 7
        a.checkpoint.wait()
        marks = stepmarks.StepMarks(job, f"{a.ctx.role}{a.ctx.index}")
        marks.set_now(7)
        vram.adopt({k: t.clone() for k, t in _state(a.flat, a.opt).items()}, pid=os.getpid())
        b = mk(CheckpointManager(job, interval=100), 999)
        b.fit(lambda m, b_: m(*b_), data, num_steps=10)
        assert b.history[0]["step"] == 8                    # resumed after 7, nothing lost
        assert b.opt.step_count == 10
        ev = [line for line in open(tmp_path / f"events-{b.ctx.role}{b.ctx.index}.jsonl") if '"restored"' in line]
        assert ev and "hbm:step7" in ev[-1]
        assert torch.equal(torch.cat([g.data for g in b.flat.groups]), torch.cat([g.data for g in ref.flat.groups]))
        assert all(torch.equal(x, y) for x, y in zip(b.opt.state_tensors().values(), ref.opt.state_tensors().values()))
        marks.close()
    finally:
        vram.release_unused()
        vram.ADOPTED_FROM.clear()
        unlink_job_segments(job)


@pytest.mark.gpu
def test_standby_warm_up_step_runs_and_frees(cuda):
    from easydl_amd.operator.standby import warm_device
    try:
        # the first call also creates what a process keeps for good (the GEMM libraries'
        # workspaces, ~300 MB under TunableOp; the ops' small module caches): a second call
        # must not keep anything more
        warm_device(cuda.index or 0)
        warm_device(cuda.index or 0)
        before = torch.cuda.memory_allocated(cuda)
        s = warm_device(cuda.index or 0)
        grown = torch.cuda.memory_allocated(cuda) - before
        s2 = warm_device(cuda.index or 0)
    finally:
        torch.cuda.tunable.enable(False)   # the warm-up switches TunableOp on, as the trainer does
    # every further call leaves the same small amount at most (no model state kept)
    assert s > 0 and s2 > 0 and grown < 32 << 20
    assert torch.cuda.memory_allocated(cuda) - before <= 2 * grown + (1 << 20)


@pytest.mark.gpu
def test_standby_full_width_warm_up_from_the_published_spec(cuda):
    from easydl_amd.operator.standby import _warm_llama, warm_device
    spec = {"model": "llama", "batch": [1, 512],
            "cfg": {"vocab_size": 4096, "dim": 1024, "n_layers": 4, "n_heads": 8, "n_kv_heads": 2, "ffn_dim": 2048,
                    "max_seq_len": 512}}
    try:
        assert _warm_llama(cuda, spec)
        assert warm_device(cuda.index or 0, spec) > 0     # first calls: a process's one-time caches
        before = torch.cuda.memory_allocated(cuda)
        assert warm_device(cuda.index or 0, spec) > 0
        after = torch.cuda.memory_allocated(cuda)
    finally:
        torch.cuda.tunable.enable(False)
    # round 4 left ~7 B per parameter of the warm-up model allocated per call (its flat buffers
    # and W^T copies: the gradient hooks formed a cycle through C++ the collector never freed);
    # now a warm-up returns to the baseline
    assert after - before < 32 << 20, (after - before) >> 20


@pytest.mark.gpu
def test_standby_warm_up_without_room_for_the_micro_batch_runs_the_widths_on_a_short_sequence(cuda):
    """A micro-batch whose one-layer pass needs more than half of the GPU: the warm-up still runs
    the layer at the worker's widths, on 512 tokens (libraries and code objects loaded while HBM
    is calm)."""
    from easydl_amd.operator.standby import _warm_llama
    spec = {"model": "llama", "batch": [256, 8192],
            "cfg": {"vocab_size": 4096, "dim": 1024, "n_layers": 4, "n_heads": 8, "n_kv_heads": 2, "ffn_dim": 2048,
                    "max_seq_len": 8192}}
    info: dict = {}
    try:
        assert _warm_llama(cuda, spec, info)
    finally:
        torch.cuda.tunable.enable(False)
    assert info["reduced_tokens"] == 512 and 2 * info["need_gb"] > info["free_gb"], info


def test_flat_params_are_collected_with_their_model():
    """No reference cycle through the parameters' C++ hook tables keeps a dropped model's
    flat buffers alive (the standby warm-up leak of round 4)."""
    import gc
    import weakref

    from easydl_amd.parallel.flat import FlatParams
    model = torch.nn.Sequential(torch.nn.Linear(8, 8), torch.nn.Linear(8, 2))
    flat = FlatParams(model)
    model(torch.randn(3, 8)).sum().backward()      # hooks have fired once
    refs = [weakref.ref(flat), weakref.ref(flat.groups[0].data), weakref.ref(model)]
    del model, flat
    gc.collect()
    assert all(r() is None for r in refs), [r() is None for r in refs]


def test_warm_spec_round_trip_and_sizing():
    from easydl_amd.models.llama import get_config
    from easydl_amd.operator.standby import _llama_warm_bytes

    class KV(dict):
        def set(self, k, v):
            self[k] = v

        def get_str(self, k):
            return self.get(k)

    kv = KV()
    assert vram.read_warm(kv, "worker0") == (False, None)
    vram.publish_warm(kv, "worker0", None)
    assert vram.read_warm(kv, "worker0") == (True, None)
    spec = {"model": "llama", "cfg": {"dim": 4096}, "batch": [1, 8192]}
    vram.publish_warm(kv, "worker0", spec)
    assert vram.read_warm(kv, "worker0") == (True, spec)
    # one Llama-3-8B layer at one 8k sequence: ~20 GB, far below what a worker leaves free
    gb = _llama_warm_bytes(get_config("llama3-8b", n_layers=1), 8192) / 2**30
    assert 10 < gb < 30


def test_hbm_resume_check_failure_stops_at_the_next_update(tmp_path):
    """The post-reap re-read of the step marks runs off the training path; if the marks moved
    (the dead worker's GPU updated the adopted state after the resume), the next optimizer
    step raises instead of training on -- and snapshots wait for the check meanwhile."""
    from types import SimpleNamespace

    from easydl_amd.ckpt.manager import CheckpointManager
    from easydl_amd.utils import stepmarks
    job = f"hbmchk{os.getpid()}"
    gone = subprocess.Popen([sys.executable, "-c", "pass"])
    gone.wait()
    m = stepmarks.StepMarks(job, "worker0")
    try:
        m.set_now(5)
        m.begin(6)                                  # the page now reads (6, 5): moved since (5, 5)
        tr = SimpleNamespace(step=0, ckpt_tag="", opt=SimpleNamespace(step_count=0, moment_origin=0),
                             load_host_state=lambda h: None)
        ck = CheckpointManager(job, interval=1)
        ck.resume_from_hbm(tr, 5, {"pid": gone.pid, "marks": (5, 5), "job": job, "slot": "worker0"})
        assert tr.step == 5 and tr.opt.step_count == 5
        t_end = time.time() + 10
        while ck.hbm_unverified() and time.time() < t_end:
            time.sleep(0.01)
        with pytest.raises(RuntimeError, match="HBM resume invalidated"):
            ck.fence()
    finally:
        m.close(unlink=True)


def test_early_hand_over_only_when_a_standby_is_ready():
    """A SIGKILLed worker is replaced before its reap only if a parked standby will take its
    place (it builds on the dead worker's HBM); a freshly started process would have to
    allocate that HBM while the dead one still holds it."""
    import signal
    from types import SimpleNamespace

    from easydl_amd.operator.reconciler import ElasticOperator, Proc
    from easydl_amd.api.spec import Resource
    child = subprocess.Popen([sys.executable, "-c", "import time; time.sleep(60)"])
    try:
        os.kill(child.pid, signal.SIGKILL)
        t_end = time.time() + 10
        from easydl_amd.utils.procfs import exit_status
        while not exit_status(child.pid) and time.time() < t_end:   # a zombie, not yet reaped
            time.sleep(0.01)
        events = []
        ready = {"v": False}
        p = Proc("job-worker-0", "worker", 0, child.pid, 0, Resource(), time.time())
        p._early_reported = True
        op = SimpleNamespace(procs={p.name: p}, history=[], restarts=0,
                             events=SimpleNamespace(emit=lambda kind, **kw: events.append(kind)),
                             _standby_ready=lambda: ready["v"], _release_gpu=lambda q: None)
        for _ in range(3):
            ElasticOperator._early_replace(op)
            time.sleep(0.12)
        assert p.state == "running" and not events          # no standby: wait for the reap
        ready["v"] = True
        for _ in range(3):
            ElasticOperator._early_replace(op)
            time.sleep(0.12)
        assert events == ["exit_early"] and p.state == "exited" and p.exit_code == -9
        assert p.name not in op.procs and op.history == [p]
    finally:
        child.wait()


def test_shared_gpu_layout_limits_hardware_queues(monkeypatch):
    """Ranks sharing a GPU get 2 hardware queues per process (the box's default is 4); a
    one-rank-per-GPU layout keeps the default, so its snapshot and engine streams keep their
    own queues -- unless the standbys (each holds a context on every GPU) push the busiest
    GPU past 8 queues."""
    from types import SimpleNamespace

    from easydl_amd.operator.reconciler import ElasticOperator
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "4")

    def env_for(gpus, standby=1):
        op = SimpleNamespace(job=SimpleNamespace(env={}, name="j", standby=0), master_port=1, run_dir="/tmp",
                             cfg=SimpleNamespace(standby=standby, gpus=gpus))
        return ElasticOperator._base_env(op)

    assert env_for([0, 0, 0])["GPU_MAX_HW_QUEUES"] == "2"
    assert env_for([0, 1, 2])["GPU_MAX_HW_QUEUES"] == "4"
    # N=8, one standby holding a context on every GPU: worker + standby = 8 queues per GPU
    assert env_for(list(range(8)))["GPU_MAX_HW_QUEUES"] == "4"
    # a second standby would put 12 per GPU: everyone, standbys included, drops to 2
    assert env_for(list(range(8)), standby=2)["GPU_MAX_HW_QUEUES"] == "2"
    monkeypatch.setenv("EDL_SHARED_GPU_HW_QUEUES", "3")
    assert env_for([0, 0])["GPU_MAX_HW_QUEUES"] == "3"
