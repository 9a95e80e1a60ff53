"""ElasticOperator reconcile logic (fake launcher) and the native supervisor (real processes)."""
import json
import os
import signal
import sys
import time

import pytest

from easydl_amd.api.spec import ElasticJob, JobResource, Resource, RoleResource, ResourceUpdation, load_specs
from easydl_amd.operator.reconciler import ElasticOperator, OperatorConfig, cu_mask_hex


class FakeExit:
    def __init__(self, pid, code=0, sig=0):
        self.pid, self.exit_code, self.signal, self.ts = pid, code, sig, time.time()


class FakeLauncher:
    def __init__(self):
        self.next = 100
        self.spawned = []
        self.killed = []
        self.pending = []

    def spawn(self, name, argv, env=None, cwd=None, log_path=None, cpus=None):
        self.next += 1
        self.spawned.append((name, self.next, env))
        return self.next

    def poll(self, timeout):
        out, self.pending = self.pending, []
        return out

    def kill(self, pid, sig=9):
        self.killed.append((pid, sig))

    def terminate(self, pid, grace_s=5):
        self.killed.append((pid, "term"))


class FakeKV:
    def __init__(self):
        self.d = {}

    def set(self, k, v):
        self.d[k] = v

    def get(self, k, default=None):
        v = self.d.get(k, default)
        if isinstance(v, str):
            try:
                return json.loads(v)
            except ValueError:
                return v
        return v

    def exists(self, k):
        return k in self.d

    def delete(self, k):
        self.d.pop(k, None)


JOB = ElasticJob.from_dict({"apiVersion": "elastic.easydl.org/v1alpha1", "kind": "ElasticJob",
                            "metadata": {"name": "j"}, "spec": {"command": "python -m x",
                                                                "worker": {"image": "img"}}})


def _op(gpus=4):
    fl = FakeLauncher()
    kv = FakeKV()
    op = ElasticOperator(JOB, "/tmp/edl_op_test", launcher=fl, cfg=OperatorConfig(gpus=list(range(gpus))), kv=kv)
    op.start()
    return op, fl, kv


def test_trainer_first_then_roles():
    op, fl, kv = _op()
    assert [s[0] for s in fl.spawned] == ["j-trainer-0"]
    op.tick()
    assert len(fl.spawned) == 1  # no JobResource yet: nothing else
    jr = JobResource("r", "j", {"worker": RoleResource(3, Resource(cpu=1, gpu=1))})
    kv.set("jobresource", json.dumps(jr.to_dict()))
    op.tick()
    names = [s[0] for s in fl.spawned[1:]]
    assert names == ["j-worker-0", "j-worker-1", "j-worker-2"]
    gpus = [s[2]["EDL_GPU"] for s in fl.spawned[1:]]
    assert gpus == ["0", "1", "2"]


def test_failed_worker_is_replaced_same_name_and_exit_reported():
    op, fl, kv = _op()
    kv.set("jobresource", json.dumps(JobResource("r", "j", {"worker": RoleResource(2, Resource(gpu=1))}).to_dict()))
    op.tick()
    pid1 = [p for n, p, _ in fl.spawned if n == "j-worker-1"][0]
    fl.pending.append(FakeExit(pid1, code=-1, sig=9))
    op.tick()
    assert kv.exists(f"ev/exit/j-worker-1:{pid1}")
    again = [(n, p) for n, p, _ in fl.spawned if n == "j-worker-1"]
    assert len(again) == 2 and again[1][1] != pid1
    assert op.restarts == 1


def test_scale_down_requests_graceful_leave_of_highest_index():
    op, fl, kv = _op()
    kv.set("jobresource", json.dumps(JobResource("r", "j", {"worker": RoleResource(3, Resource(gpu=1))},
                                                 version=1).to_dict()))
    op.tick()
    kv.set("jobresource", json.dumps(JobResource("r", "j", {"worker": RoleResource(2, Resource(gpu=1))},
                                                 version=2).to_dict()))
    op.tick()
    pid2 = [p for n, p, _ in fl.spawned if n == "j-worker-2"][0]
    assert kv.exists(f"rdzv/leave/j-worker-2:{pid2}")


def test_resource_updation_replaces_named_process_with_merged_resource():
    op, fl, kv = _op(gpus=2)
    jr = JobResource("r", "j", {"worker": RoleResource(2, Resource(cpu=2, memory=1024, gpu=1))}, version=1)
    kv.set("jobresource", json.dumps(jr.to_dict()))
    op.tick()
    jr.version = 2
    jr.resource_updation = [ResourceUpdation("j-worker-0", Resource(cpu=8, cu=128))]
    kv.set("jobresource", json.dumps(jr.to_dict()))
    op.tick()
    old = [p for n, p, _ in fl.spawned if n == "j-worker-0"][0]
    assert kv.exists(f"rdzv/leave/j-worker-0:{old}")
    # both GPUs busy: the replacement waits for the old incarnation to exit
    assert len([n for n, _, _ in fl.spawned if n == "j-worker-0"]) == 1
    fl.pending.append(FakeExit(old, 0))
    op.tick()
    news = [(p, e) for n, p, e in fl.spawned if n == "j-worker-0"]
    assert len(news) == 2
    env = news[1][1]
    assert env["EDL_CU_MASK"] == cu_mask_hex(128) and env["EDL_GPU"] == "0"


def test_clean_exit_completes_job():
    op, fl, kv = _op()
    kv.set("jobresource", json.dumps(JobResource("r", "j", {"worker": RoleResource(2, Resource(gpu=1))}).to_dict()))
    op.tick()
    for n, p, _ in list(fl.spawned):
        if n.startswith("j-worker"):
            fl.pending.append(FakeExit(p, 0))
    op.tick()
    assert op.done


def test_cu_mask_spreads_over_xcds():
    m = int(cu_mask_hex(8), 16)
    assert bin(m).count("1") == 8
    assert {b % 8 for b in range(256) if m >> b & 1} == set(range(8))
    assert bin(int(cu_mask_hex(256), 16)).count("1") == 256


def test_reference_yaml_roundtrip():
    ref = """
apiVersion: elastic.easydl.org/v1alpha1
kind: ElasticJob
metadata:
  name: elastic-deepctr-job
spec:
  command: "python -m model_zoo.iris.dnn_estimator"
  image:
  parameter_server:
    image: elasticdl:iris_estimator
  worker:
    image: elasticdl:iris_estimator
  evaluator:
    image: elasticdl:iris_estimator
---
apiVersion: elastic.easydl.org/v1alpha1
kind: JobResource
metadata:
  name: "elastic-training-resource"
spec:
  selector:
    name: elastic-deepctr-job  // Job Name
  parameter_server:
    replicas: 4
    resource:
      cpu: 4
      memory: 4096
      disk: 8192
      gpu: 1
  worker:
    replicas: 4
    resource: {cpu: 4, memory: 4096, disk: 8192, gpu: 1}
  evaluator:
    replicas: 1
    resource: {cpu: 4, memory: 4096, disk: 8192, gpu: 1}
  resource_updation:
    - name: "elastic-deepctr-job-ps-0"
      resource: {cpu: 8, memory: 8192}
    - name: "elastic-deepctr-job-ps-1"
      resource: {cpu: 16, memory: 8192}
"""
    job, jr = load_specs(ref)
    assert job.name == "elastic-deepctr-job" and job.mode == "ps"
    assert set(job.roles) == {"parameter_server", "worker", "evaluator"}
    assert jr.selector == "elastic-deepctr-job"
    assert jr.replicas("parameter_server") == 4 and jr.roles["worker"].resource.memory == 4096
    assert [u.name for u in jr.resource_updation] == ["elastic-deepctr-job-ps-0", "elastic-deepctr-job-ps-1"]
    assert jr.resource_updation[1].resource.cpu == 16 and jr.resource_updation[1].resource.gpu is None
    merged = jr.roles["parameter_server"].resource.merged(jr.resource_updation[0].resource)
    assert merged.cpu == 8 and merged.gpu == 1 and merged.disk == 8192
    # round trip
    jr2 = JobResource.from_dict(jr.to_dict())
    assert jr2.to_dict() == jr.to_dict()


def test_native_supervisor_exit_events(tmp_path):
    from easydl_amd.operator.supervisor import Supervisor
    sup = Supervisor()
    try:
        t0 = time.time()
        p_ok = sup.spawn("ok", [sys.executable, "-c", "print('hi')"], env=dict(os.environ),
                         log_path=str(tmp_path / "ok.log"))
        p_bad = sup.spawn("bad", [sys.executable, "-c", "import sys; sys.exit(7)"], env=dict(os.environ))
        p_sleep = sup.spawn("sleep", ["sleep", "30"], cpus=[0])
        seen = {}
        t_end = time.time() + 20
        while len(seen) < 2 and time.time() < t_end:
            for e in sup.poll(0.5):
                seen[e.name] = e
        assert seen["ok"].ok and seen["bad"].exit_code == 7
        assert "hi" in open(tmp_path / "ok.log").read()
        sup.kill(p_sleep, signal.SIGKILL)
        t_kill = time.time()
        ev = []
        while not ev and time.time() < t_end:
            ev = sup.poll(0.5)
        assert ev[0].name == "sleep" and ev[0].signal == signal.SIGKILL
        assert ev[0].ts - t_kill < 0.5  # pidfd: near-immediate detection
        with pytest.raises(OSError):
            sup.spawn("nope", ["/nonexistent/binary"])
    finally:
        sup.close()
