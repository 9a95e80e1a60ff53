"""Multi-process elastic training on CPU/gloo: static world, kill-a-worker shrink,
scale-up join.  Processes are real (subprocess), the store is a real TCPStore."""
import json
import os
import socket
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "helpers", "elastic_worker.py")


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _env(tmp, idx, extra):
    e = dict(os.environ)
    e.update({"EDL_JOB": "t", "EDL_ROLE": "worker", "EDL_INDEX": str(idx), "EDL_RUN_DIR": str(tmp),
              "TEST_OUT": str(tmp / f"res{idx}.json"), "OMP_NUM_THREADS": "1", "PYTHONPATH": ROOT})
    e.pop("WORLD_SIZE", None)
    e.update(extra)
    return e


def _start_master(tmp, port, mn, mx, window=0.3, initial=0, granule=1):
    return subprocess.Popen([sys.executable, "-m", "easydl_amd.master.main", "--job", "t", "--port", str(port),
                             "--min", str(mn), "--max", str(mx), "--join-window", str(window),
                             "--initial", str(initial), "--granule", str(granule),
                             "--run-dir", str(tmp)], cwd=ROOT, env=dict(os.environ, PYTHONPATH=ROOT),
                            stdout=subprocess.PIPE, stderr=subprocess.STDOUT)


def _results(tmp, idxs):
    return {i: json.load(open(tmp / f"res{i}.json")) for i in idxs}


def _wait(procs, timeout=240):
    t_end = time.time() + timeout
    codes = {}
    for i, p in procs.items():
        try:
            codes[i] = p.wait(timeout=max(1, t_end - time.time()))
        except subprocess.TimeoutExpired:
            p.kill()
            codes[i] = "timeout"
    return codes


@pytest.mark.slow
def test_torchrun_style_static_world(tmp_path):
    port = free_port()
    procs = {}
    for i in range(2):
        env = _env(tmp_path, i, {"RANK": str(i), "WORLD_SIZE": "2", "MASTER_ADDR": "127.0.0.1",
                                 "MASTER_PORT": str(port), "TEST_STEPS": "5", "TEST_GB": "4"})
        env.pop("EDL_INDEX")
        procs[i] = subprocess.Popen([sys.executable, WORKER], env=env, cwd=ROOT)
    codes = _wait(procs)
    assert codes == {0: 0, 1: 0}, codes
    r = _results(tmp_path, [0, 1])
    assert r[0]["hash"] == r[1]["hash"]
    assert r[0]["step"] == 5 and r[0]["worlds"] == [2] * 5


@pytest.mark.slow
def test_kill_worker_shrinks_and_continues(tmp_path):
    port = free_port()
    m = _start_master(tmp_path, port, 1, 3, initial=3)
    try:
        procs = {}
        for i in range(3):
            env = _env(tmp_path, i, {"EDL_MASTER_ADDR": "127.0.0.1", "EDL_MASTER_PORT": str(port),
                                     "TEST_STEPS": "8", "TEST_GB": "6",
                                     "EDL_FAULT": "kill@step=3,index=2"})
            procs[i] = subprocess.Popen([sys.executable, WORKER], env=env, cwd=ROOT)
        # emulate the operator's supervisor: report the exit event
        t_end = time.time() + 240
        reported = False
        while time.time() < t_end and not reported:
            rc = procs[2].poll()
            if rc is not None:
                from easydl_amd.master.store import KV, make_tcp_store
                kv = KV(make_tcp_store("127.0.0.1", port, False), "edl/t")
                node = [n for n in (kv.get_str("rdzv/joined") or "").split(",") if n.startswith("t-worker-2:")][0]
                kv.set(f"ev/exit/{node}", json.dumps({"code": rc}))
                reported = True
            time.sleep(0.05)
        codes = _wait({0: procs[0], 1: procs[1]})
        assert codes == {0: 0, 1: 0}, codes
        r = _results(tmp_path, [0, 1])
        assert r[0]["hash"] == r[1]["hash"], "survivors diverged"
        assert r[0]["step"] == 8
        assert r[0]["worlds"][0] == 3 and r[0]["worlds"][-1] == 2
        from easydl_amd.utils.events import read_events, ttr_breakdown
        ttr = ttr_breakdown(read_events(str(tmp_path)))
        assert ttr is not None and ttr["ttr_s"] is not None and ttr["ttr_s"] < 60, ttr
    finally:
        m.terminate()


@pytest.mark.slow
def test_scale_up_joiner_receives_state(tmp_path):
    port = free_port()
    m = _start_master(tmp_path, port, 1, 3, window=0.2)
    try:
        procs = {}
        for i in range(2):
            env = _env(tmp_path, i, {"EDL_MASTER_ADDR": "127.0.0.1", "EDL_MASTER_PORT": str(port),
                                     "TEST_STEPS": "30", "TEST_GB": "6", "TEST_STEP_SLEEP": "0.25"})
            procs[i] = subprocess.Popen([sys.executable, WORKER], env=env, cwd=ROOT)
        time.sleep(4.0)
        env = _env(tmp_path, 2, {"EDL_MASTER_ADDR": "127.0.0.1", "EDL_MASTER_PORT": str(port),
                                 "TEST_STEPS": "30", "TEST_GB": "6", "TEST_STEP_SLEEP": "0.25"})
        procs[2] = subprocess.Popen([sys.executable, WORKER], env=env, cwd=ROOT)
        codes = _wait(procs)
        assert codes == {0: 0, 1: 0, 2: 0}, codes
        r = _results(tmp_path, [0, 1, 2])
        assert r[0]["hash"] == r[1]["hash"] == r[2]["hash"]
        assert 3 in r[0]["worlds"], r[0]["worlds"]
        assert r[2]["step"] == 30
        # a process joining a running job warms up before announcing itself; whichever of
        # the two initial workers formed the first (world-1) epoch never does (the other
        # may have found that epoch running, depending on start-up timing)
        from easydl_amd.utils.events import read_events
        warm = {e.get("proc") for e in read_events(str(tmp_path)) if e["kind"] == "prejoin_warmup"}
        assert "worker2" in warm and len(warm & {"worker0", "worker1"}) <= 1, warm
    finally:
        m.terminate()


def _report_exit(port, idx, rc):
    from easydl_amd.master.store import KV, make_tcp_store
    kv = KV(make_tcp_store("127.0.0.1", port, False), "edl/t")
    node = [n for n in (kv.get_str("rdzv/joined") or "").split(",") if n.startswith(f"t-worker-{idx}:")][0]
    kv.set(f"ev/exit/{node}", json.dumps({"code": rc}))


@pytest.mark.slow
def test_tp2_dp2_static_replicas_agree(tmp_path):
    """DP x TP mesh (tp=2, dp=2): TP ranks of a replica see the same batch, DP
    replicas of each shard stay bit-identical, all ranks report one loss."""
    port = free_port()
    m = _start_master(tmp_path, port, 2, 4, initial=4, granule=2)
    try:
        procs = {}
        for i in range(4):
            env = _env(tmp_path, i, {"EDL_MASTER_ADDR": "127.0.0.1", "EDL_MASTER_PORT": str(port),
                                     "TEST_STEPS": "6", "TEST_GB": "4", "EDL_TP": "2"})
            procs[i] = subprocess.Popen([sys.executable, WORKER], env=env, cwd=ROOT)
        codes = _wait(procs)
        assert codes == {0: 0, 1: 0, 2: 0, 3: 0}, codes
        r = _results(tmp_path, range(4))
        by_tp = {}
        for x in r.values():
            assert x["step"] == 6 and x["worlds"] == [4] * 6
            by_tp.setdefault(x["tp_rank"], set()).add(x["hash"])
        assert sorted(by_tp) == [0, 1] and all(len(v) == 1 for v in by_tp.values()), by_tp
        assert by_tp[0] != by_tp[1]
        by_dp = {}
        for x in r.values():  # the TP ranks of one replica compute one loss
            by_dp.setdefault(x["dp_rank"], set()).add(round(x["loss"], 6))
        assert sorted(by_dp) == [0, 1] and all(len(v) == 1 for v in by_dp.values()), by_dp
    finally:
        m.terminate()


@pytest.mark.slow
def test_tp2_kill_worker_keeps_shards(tmp_path):
    """tp=2 world 4 -> a worker dies -> world 2 (granule 2): the survivors that
    keep their TP rank continue without restore; the spare exits cleanly."""
    port = free_port()
    m = _start_master(tmp_path, port, 2, 4, initial=4, granule=2)
    try:
        procs = {}
        for i in range(4):
            env = _env(tmp_path, i, {"EDL_MASTER_ADDR": "127.0.0.1", "EDL_MASTER_PORT": str(port),
                                     "TEST_STEPS": "8", "TEST_GB": "4", "EDL_TP": "2",
                                     "EDL_FAULT": "kill@step=3,index=3"})
            procs[i] = subprocess.Popen([sys.executable, WORKER], env=env, cwd=ROOT)
        t_end = time.time() + 240
        while time.time() < t_end:
            rc = procs[3].poll()
            if rc is not None:
                _report_exit(port, 3, rc)
                break
            time.sleep(0.05)
        codes = _wait({i: procs[i] for i in range(3)})
        assert codes == {0: 0, 1: 0, 2: 0}, codes
        r = _results(tmp_path, range(3))
        done = [x for x in r.values() if x["step"] == 8]
        assert len(done) == 2 and {x["tp_rank"] for x in done} == {0, 1}, r
        assert done[0]["worlds"][0] == 4 and done[0]["worlds"][-1] == 2
        from easydl_amd.utils.events import read_events
        ev = read_events(str(tmp_path))
        assert not [e for e in ev if e["kind"] == "restored"], "no restore needed: shards survived"
        assert [e for e in ev if e["kind"] == "finished_waiting"], "spare worker did not exit via train/done"
    finally:
        m.terminate()


@pytest.mark.slow
def test_tp_shard_lost_restores_from_snapshot(tmp_path):
    """tp=2 = world (no DP replica): a dead worker's shard has no live holder;
    after the operator-style replacement joins, BOTH ranks roll back to the
    newest common in-memory snapshot and finish."""
    from easydl_amd.ckpt.manager import unlink_job_segments
    job = f"tpck{os.getpid()}"
    unlink_job_segments(job)
    port = free_port()
    m = _start_master(tmp_path, port, 2, 2, initial=2, granule=2)
    try:
        procs = {}
        base = {"EDL_MASTER_ADDR": "127.0.0.1", "EDL_MASTER_PORT": str(port), "TEST_STEPS": "8", "TEST_GB": "4",
                "EDL_TP": "2", "TEST_CKPT": "2", "TEST_CKPT_JOB": job}
        for i in range(2):
            procs[i] = subprocess.Popen([sys.executable, WORKER],
                                        env=_env(tmp_path, i, dict(base, EDL_FAULT="kill@step=5,index=1")), cwd=ROOT)
        t_end = time.time() + 240
        while time.time() < t_end:
            rc = procs[1].poll()
            if rc is not None:
                _report_exit(port, 1, rc)
                break
            time.sleep(0.05)
        env = _env(tmp_path, 1, dict(base, EDL_GENERATION="1", TEST_OUT=str(tmp_path / "res1b.json")))
        procs["r"] = subprocess.Popen([sys.executable, WORKER], env=env, cwd=ROOT)
        codes = _wait({0: procs[0], "r": procs["r"]})
        assert codes == {0: 0, "r": 0}, codes
        a, b = json.load(open(tmp_path / "res0.json")), json.load(open(tmp_path / "res1b.json"))
        assert a["step"] == b["step"] == 8 and {a["tp_rank"], b["tp_rank"]} == {0, 1}
        from easydl_amd.utils.events import read_events
        rs = [e for e in read_events(str(tmp_path)) if e["kind"] == "restored"]
        assert len(rs) == 2 and {e["step"] for e in rs} == {4}, rs
    finally:
        m.terminate()
        unlink_job_segments(job)


def test_snapshot_fenced_before_a_broadcast_rewrites_state():
    """_fence_snapshot_before_overwrite: the in-flight snapshot D2H is fenced exactly when
    this rank's buffers are about to change (receiver, or any non-source rank of the
    xGMI-only broadcast, which zero-fills), never on the source or an RCCL holder."""
    from types import SimpleNamespace

    import torch

    from easydl_amd.trainer.elastic import ElasticTrainer

    calls = []
    ck = SimpleNamespace(fence=lambda: calls.append(1))
    me = SimpleNamespace(checkpoint=ck, device=torch.device("cuda", 0))
    fn = ElasticTrainer._fence_snapshot_before_overwrite
    cases = [  # (rank, src, holder, backend) -> fenced?
        (0, 0, True, "rccl", False),    # the source
        (1, 0, True, "rccl", False),    # holder receiving identical bytes
        (1, 0, False, "rccl", True),    # receiver: buffers change
        (1, 0, True, "xgmi", True),     # xGMI-only broadcast zero-fills non-source ranks
        (0, 0, True, "xgmi", False),
    ]
    for rank, src, holder, backend, want in cases:
        calls.clear()
        fn(me, SimpleNamespace(rank=rank, backend=backend), src, holder)
        assert bool(calls) == want, (rank, src, holder, backend)
    calls.clear()
    fn(SimpleNamespace(checkpoint=None, device=torch.device("cuda", 0)), SimpleNamespace(rank=1, backend="xgmi"), 0,
       False)
    fn(SimpleNamespace(checkpoint=ck, device=torch.device("cpu")), SimpleNamespace(rank=1, backend="xgmi"), 0, False)
    assert not calls   # no checkpoint manager / CPU state: nothing to fence


@pytest.mark.slow
def test_runtime_plan_switches_every_rank_at_one_step(tmp_path):
    """Brain runtime knobs (master/planner.py): one document per plan version; ranks
    adopt the agreed version at epoch entry and switch at one committed step."""
    from easydl_amd.master.store import KV, make_tcp_store
    from easydl_amd.utils.events import read_events
    port = free_port()
    m = _start_master(tmp_path, port, 1, 2, initial=2)
    try:
        kv = KV(make_tcp_store("127.0.0.1", port, False), "edl/t")
        kv.set("plan/runtime/1", json.dumps({"bucket_mb": 0.1, "ckpt_interval": None, "allreduce": None}))
        kv.add("plan/version", 1)
        procs = {}
        for i in range(2):
            env = _env(tmp_path, i, {"EDL_MASTER_ADDR": "127.0.0.1", "EDL_MASTER_PORT": str(port),
                                     "TEST_STEPS": "40", "TEST_GB": "4", "TEST_STEP_SLEEP": "0.1"})
            procs[i] = subprocess.Popen([sys.executable, WORKER], env=env, cwd=ROOT)

        def applied(mb):
            return {e.get("proc"): e.get("step") for e in read_events(str(tmp_path))
                    if e["kind"] == "plan_bucket_mb" and e.get("mb") == mb}

        t_end = time.time() + 120
        while len(applied(0.1)) < 2 and time.time() < t_end:
            time.sleep(0.1)
        assert len(applied(0.1)) == 2, "version 1 not adopted at epoch entry"
        kv.set("plan/runtime/2", json.dumps({"bucket_mb": 0.05, "ckpt_interval": None, "allreduce": None}))
        kv.add("plan/version", 1)
        codes = _wait(procs)
        assert codes == {0: 0, 1: 0}, codes
        r = _results(tmp_path, [0, 1])
        assert r[0]["hash"] == r[1]["hash"]
        assert r[0]["bucket_mb"] == r[1]["bucket_mb"] == 0.05 and r[0]["plan_version"] == r[1]["plan_version"] == 2
        steps = applied(0.05)
        assert len(steps) == 2 and len(set(steps.values())) == 1, steps   # the same committed step
    finally:
        m.terminate()


@pytest.mark.slow
def test_brain_plan_loop_retunes_buckets_on_running_workers(tmp_path):
    """The whole Brain loop on a live job: the master asks the Brain for a startup plan
    (bucket size in plan/runtime/1), collects the workers' step metrics, the Brain's
    bucket autotune re-plans, and both workers switch to the new bucket size at one
    committed step with identical weights."""
    from easydl_amd.utils.events import read_events
    spec = {"apiVersion": "edl.mi355x/v1", "kind": "ElasticJob", "metadata": {"name": "t"},
            "spec": {"command": "python -m x", "min_workers": 2, "max_workers": 2,
                     "features": {"model": "tiny", "params": 2e5, "mode": "allreduce", "min_workers": 2,
                                  "max_workers": 2}}}
    jf = tmp_path / "job.json"
    jf.write_text(json.dumps(spec))
    port = free_port()
    m = subprocess.Popen([sys.executable, "-m", "easydl_amd.master.main", "--job", "t", "--port", str(port),
                          "--min", "1", "--max", "2", "--join-window", "0.3", "--initial", "2",
                          "--run-dir", str(tmp_path), "--job-spec", str(jf), "--plan-period", "0.5"],
                         cwd=ROOT, env=dict(os.environ, PYTHONPATH=ROOT), stdout=subprocess.PIPE,
                         stderr=subprocess.STDOUT)
    try:
        procs = {}
        for i in range(2):
            env = _env(tmp_path, i, {"EDL_MASTER_ADDR": "127.0.0.1", "EDL_MASTER_PORT": str(port),
                                     "TEST_STEPS": "60", "TEST_GB": "4", "TEST_STEP_SLEEP": "0.05"})
            procs[i] = subprocess.Popen([sys.executable, WORKER], env=env, cwd=ROOT)
        codes = _wait(procs)
        assert codes == {0: 0, 1: 0}, codes
        r = _results(tmp_path, [0, 1])
        assert r[0]["hash"] == r[1]["hash"]
        ev = read_events(str(tmp_path))
        kinds = {e["kind"] for e in ev}
        assert "startup_plan" in kinds and "replan" in kinds, kinds
        switched = {}
        for e in ev:
            if e["kind"] == "plan_bucket_mb":
                switched.setdefault(e.get("proc"), []).append((e["step"], e["mb"]))
        assert set(switched) == {"worker0", "worker1"}, switched
        assert switched["worker0"] == switched["worker1"], switched      # same sizes at the same steps
        assert len(switched["worker0"]) >= 2, switched                   # startup plan + >= 1 autotune move
        assert r[0]["plan_version"] == r[1]["plan_version"] >= 2
    finally:
        m.terminate()


@pytest.mark.slow
def test_tp2_dp3_replacement_receives_shard_from_every_holder(tmp_path):
    """tp=2, dp=3 (world 6) -> one worker dies -> world 4 (granule 2: one survivor parks as
    a spare) -> a replacement process arrives -> world 6.  The two ranks that need a shard
    (the replacement and the stale spare) receive it from BOTH holders of their DP group at
    once (multi-source transfer_state), bit-exact: every DP replica of
    each shard ends identical."""
    port = free_port()
    m = _start_master(tmp_path, port, 2, 6, initial=6, granule=2, window=0.3)
    try:
        # 60 steps of >= 0.2 s: the world-4 epoch must still be training when the replacement (a fresh
        # interpreter, slow to import under a loaded CPU tier) joins, or the job ends at world 4
        common = {"EDL_MASTER_ADDR": "127.0.0.1", "EDL_MASTER_PORT": str(port), "TEST_STEPS": "60",
                  "TEST_GB": "6", "EDL_TP": "2", "TEST_STEP_SLEEP": "0.2"}
        procs = {}
        for i in range(6):
            extra = dict(common, EDL_FAULT="kill@step=3,index=5") if i == 5 else common
            procs[i] = subprocess.Popen([sys.executable, WORKER], env=_env(tmp_path, i, extra), cwd=ROOT)
        t_end = time.time() + 120
        while time.time() < t_end and procs[5].poll() is None:
            time.sleep(0.05)
        _report_exit(port, 5, procs[5].poll())
        from easydl_amd.utils.events import read_events
        t_end = time.time() + 60        # the world-4 epoch forms and trains a few steps
        while time.time() < t_end and not any(e["kind"] == "epoch_formed" and e.get("world") == 4
                                              for e in read_events(str(tmp_path))):
            time.sleep(0.1)
        time.sleep(1.0)
        env = _env(tmp_path, 6, dict(common, TEST_OUT=str(tmp_path / "res6.json")))
        procs[6] = subprocess.Popen([sys.executable, WORKER], env=env, cwd=ROOT)
        codes = _wait({i: p for i, p in procs.items() if i != 5})
        assert all(v == 0 for v in codes.values()), codes
        r = _results(tmp_path, [0, 1, 2, 3, 4, 6])
        assert all(x["step"] == 60 for x in r.values()), {i: (x["step"], x["worlds"]) for i, x in r.items()}
        assert 6 in r[6]["worlds"] and any(4 in x["worlds"] for x in r.values()), {i: x["worlds"] for i, x in r.items()}
        by_tp = {}
        for x in r.values():
            by_tp.setdefault(x["tp_rank"], set()).add(x["hash"])
        assert sorted(by_tp) == [0, 1] and all(len(v) == 1 for v in by_tp.values()), by_tp
        sends = [e for e in read_events(str(tmp_path)) if e["kind"] == "state_broadcast" and e.get("group") == "dp"]
        assert sends and max(e.get("sources", 1) for e in sends) == 2, sends
    finally:
        m.terminate()


def test_retire_releases_an_aborted_engine_off_thread():
    """An aborted epoch's xGMI engine is released (close_after_abort) on a background thread;
    a healthy epoch's engine is left to the normal shutdown."""
    import threading as _th

    from easydl_amd.trainer.elastic import _retire

    class Eng:
        def __init__(self):
            self.closed = _th.Event()

        def close_after_abort(self):
            self.closed.set()

    class C:
        def __init__(self, aborted):
            self.aborted, self.xgmi, self.data, self.ctrl = aborted, Eng(), None, None

    live, dead = C(False), C(True)
    e_live, e_dead = live.xgmi, dead.xgmi
    _retire(live)
    _retire(dead)
    assert e_dead.closed.wait(5) and dead.xgmi is None
    assert live.xgmi is e_live and not e_live.closed.is_set()


@pytest.mark.slow
def test_tp_shard_restore_keeps_moments_when_fp32_slots_do_not_fit(tmp_path):
    """Config 5's host-DRAM squeeze on the CPU tier: the per-rank budget (EDL_CKPT_HOST_GB) holds
    two full snapshot slots only with bf16 moments (two fp32-moment slots would force LEAN, i.e.
    a restore that restarts Adam).  moment_dtype=auto picks bf16 moments; the TP shard that loses
    its only holder restores weights AND moments, and the run ends bit-identical -- every weight,
    master and moment byte -- to an uninterrupted run of the same configuration."""
    from easydl_amd.ckpt.manager import unlink_job_segments
    from easydl_amd.models.llama import get_config
    cfg = get_config("llama-tiny", n_layers=1, dim=64, n_heads=4, n_kv_heads=2, ffn_dim=128, vocab_size=128)
    # one TP rank's shard of that model (~half the parameters): 12 B/param fp32-moment slots vs 8 B/param
    n = sum(p.numel() for p in __import__("easydl_amd.models.llama", fromlist=["Llama"]).Llama(cfg).parameters())
    budget_gb = 2 * (n / 2 * 10) / 2**30              # between 2 x 8 B and 2 x 12 B per shard parameter

    def run(sub, fault):
        job = f"tpm{sub}{os.getpid()}"
        unlink_job_segments(job)
        out = tmp_path / sub
        out.mkdir()
        port = free_port()
        m = _start_master(out, port, 2, 2, initial=2, granule=2)
        try:
            base = {"EDL_MASTER_ADDR": "127.0.0.1", "EDL_MASTER_PORT": str(port), "TEST_STEPS": "8", "TEST_GB": "4",
                    "EDL_TP": "2", "TEST_CKPT": "2", "TEST_CKPT_JOB": job, "TEST_MOMENTS": "auto",
                    "EDL_CKPT_HOST_GB": repr(budget_gb)}
            procs = {i: subprocess.Popen([sys.executable, WORKER], cwd=ROOT, env=_env(
                out, i, dict(base, EDL_FAULT="kill@step=5,index=1" if (fault and i == 1) else ""))) for i in range(2)}
            if fault:
                t_end = time.time() + 240
                while time.time() < t_end:
                    rc = procs[1].poll()
                    if rc is not None:
                        _report_exit(port, 1, rc)
                        break
                    time.sleep(0.05)
                env = _env(out, 1, dict(base, EDL_GENERATION="1", TEST_OUT=str(out / "res1.json")))
                procs[1] = subprocess.Popen([sys.executable, WORKER], env=env, cwd=ROOT)
            codes = _wait(procs)
            assert codes == {0: 0, 1: 0}, codes
            res = _results(out, [0, 1])
            from easydl_amd.utils.events import read_events
            return res, read_events(str(out))
        finally:
            m.terminate()
            unlink_job_segments(job)

    ref, _ = run("ref", False)
    got, ev = run("kill", True)
    for r in list(ref.values()) + list(got.values()):
        assert r["step"] == 8 and r["moment_dtype"] == "bfloat16" and r["snapshot_mode"] == "full", r
    md = [e for e in ev if e["kind"] == "moment_dtype" and "budget_bytes" in e]
    assert md and all(2 * e["full_fp32_bytes"] > e["budget_bytes"] >= 2 * e["full_bf16_bytes"] for e in md), md
    rs = [e for e in ev if e["kind"] == "restored"]
    assert len(rs) == 2 and {e["step"] for e in rs} == {4}, rs
    by_tp = lambda res: {r["tp_rank"]: r["state_hash"] for r in res.values()}  # noqa: E731
    assert by_tp(got) == by_tp(ref)          # weights, fp32 master and bf16 moments: bit for bit
