"""Parameter-server mode on CPU: in-process PS/client, and the BASELINE config-1
job (MNIST MLP, 1 PS + 2 workers + evaluator) through the operator, with a
worker kill (training continues, data requeued) and a PS kill (replacement
restores the shard from its /dev/shm snapshot)."""
import glob
import json
import os
import signal
import subprocess
import sys
import textwrap
import threading
import time

import pytest
import torch

from easydl_amd.models.mlp import MLP, SyntheticMNIST, accuracy
from easydl_amd.ps.client import PSClient, partition, shard_of
from easydl_amd.ps.server import ParameterServer

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_partition_balanced_and_deterministic():
    sizes = [("a", 100), ("b", 90), ("c", 50), ("d", 40), ("e", 10)]
    p = partition(sizes, 2)
    assert p == partition(list(reversed(sizes)), 2)
    load = [sum(n for k, n in sizes if p[k] == i) for i in range(2)]
    assert abs(load[0] - load[1]) <= 20


@pytest.mark.parametrize("mode", ["async", "sync"])
def test_ps_inprocess_training(mode):
    torch.manual_seed(0)
    data = SyntheticMNIST(4000)
    ref = MLP()
    servers = [ParameterServer(i, shard_of(ref, 2, i), lr=3e-3, mode=mode,
                               expected_workers=lambda: 2).start() for i in range(2)]
    try:
        addrs = {i: (s.host, s.port) for i, s in enumerate(servers)}

        def work(wid):
            m = MLP()
            c = PSClient(2, lambda i: addrs[i], f"w{wid}")
            c.bind(m)
            for step in range(40):
                c.pull(m)
                m.zero_grad()
                idx = range((step * 2 + wid) * 32 % 3000, (step * 2 + wid) * 32 % 3000 + 32)
                m(*data.batch(idx)).backward()
                c.push(m, step)
            c.close()

        ts = [threading.Thread(target=work, args=(w,)) for w in range(2)]
        [t.start() for t in ts]
        [t.join(60) for t in ts]
        m = MLP()
        c = PSClient(2, lambda i: addrs[i], "eval")
        c.bind(m)
        vers = c.pull(m)
        assert accuracy(m, data) > 0.6
        if mode == "sync":
            assert vers == [40, 40]      # one update per round of 2 workers
        else:
            assert vers == [80, 80]      # every push applied
    finally:
        for s in servers:
            s.stop()


@pytest.mark.slow
def test_mnist_ps_job_with_worker_and_ps_failures(tmp_path):
    spec = tmp_path / "job.yaml"
    spec.write_text(textwrap.dedent("""
        apiVersion: elastic.easydl.org/v1alpha1
        kind: ElasticJob
        metadata: {name: mnist}
        spec:
          command: "python -m easydl_amd.examples.mnist"
          parameter_server: {image: local}
          worker: {image: local}
          evaluator: {image: local}
          env: {EDL_SAMPLES: "12000", EDL_SHARD: "512", EDL_BATCH: "64", EDL_FAULT: "kill@step=20,index=1"}
        ---
        apiVersion: elastic.easydl.org/v1alpha1
        kind: JobResource
        metadata: {name: mnist-resource}
        spec:
          selector: {name: mnist}
          parameter_server: {replicas: 1, resource: {cpu: 1, memory: 1024, gpu: 0}}
          worker: {replicas: 2, resource: {cpu: 1, memory: 1024, gpu: 0}}
          evaluator: {replicas: 1, resource: {cpu: 1, memory: 1024, gpu: 0}}
        """))
    run = tmp_path / "run"
    proc = subprocess.Popen([sys.executable, "-m", "easydl_amd.cli", "submit", str(spec), "--gpus", "",
                             "--run-dir", str(run), "--timeout", "240"], cwd=ROOT,
                            stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                            env=dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1"))
    # kill the PS once it has published its address and made progress
    from easydl_amd.master.store import KV, make_tcp_store
    first = json.loads(proc.stdout.readline())
    kv = KV(make_tcp_store("127.0.0.1", first["master_port"], False), "edl/mnist")
    t_end = time.time() + 120
    killed = False
    while time.time() < t_end and not killed:
        a = kv.get("ps/addr/0")
        if a and kv.counter("data/done") >= 3:
            os.kill(int(a["pid"]), signal.SIGKILL)
            killed = True
        time.sleep(0.1)
    out, _ = proc.communicate(timeout=300)
    assert proc.returncode == 0, out[-4000:]
    assert killed
    ev = [json.loads(l) for f in glob.glob(str(run / "events-*.jsonl")) for l in open(f)]
    kinds = [e["kind"] for e in ev]
    assert "ps_restored" in kinds, "replacement PS did not restore its shard"
    assert "data_requeued" in kinds or any(e["kind"] == "exit" and e.get("signal") == 9 for e in ev)
    done = {e["shard"] for e in ev if e["kind"] == "shard_done"}
    assert done == set(range((12000 + 511) // 512)), sorted(done)   # every shard exactly covered
    evals = [e for e in ev if e["kind"] == "eval"]
    assert evals and evals[-1]["acc"] > 0.6, evals[-1:]


@pytest.mark.parametrize("mode", ["async", "sync"])
def test_deepfm_sparse_tables_on_ps(mode):
    """DeepFM with row-striped embedding tables: workers hold no table, pull only the
    rows a batch touches, push de-duplicated row grads; the PS applies lazy Adagrad."""
    from easydl_amd.models.deepctr import DeepFM, SyntheticCTR, auc
    from easydl_amd.ps.embedding import table_shard_spec
    torch.manual_seed(0)
    vocab = 500
    data = SyntheticCTR(40000, vocab=vocab)
    ref = DeepFM(vocab=vocab, hidden=(64, 64))
    servers = [ParameterServer(i, shard_of(ref, 2, i), lr=2e-3, mode=mode, expected_workers=lambda: 2,
                               tables=table_shard_spec(ref, 2, i), sparse_optimizer="adagrad",
                               sparse_lr=0.05).start() for i in range(2)]
    assert servers[0].tables["emb"].rows == 26 * vocab // 2
    try:
        addrs = {i: (s.host, s.port) for i, s in enumerate(servers)}
        base = None

        def work(wid):
            m = DeepFM(vocab=vocab, hidden=(64, 64))
            c = PSClient(2, lambda i: addrs[i], f"w{wid}")
            c.bind(m)
            assert m.emb.weight is None           # the table lives on the PS only
            for step in range(60):
                c.pull(m)
                m.zero_grad()
                b0 = (step * 2 + wid) * 256
                m(*data.batch(range(b0, b0 + 256))).backward()
                c.push(m, step)
            c.close()

        m = DeepFM(vocab=vocab, hidden=(64, 64))
        c = PSClient(2, lambda i: addrs[i], "eval")
        c.bind(m)
        c.pull(m)
        base = auc(m, data)
        ts = [threading.Thread(target=work, args=(w,)) for w in range(2)]
        [t.start() for t in ts]
        [t.join(120) for t in ts]
        vers = c.pull(m)
        after = auc(m, data)
        assert after > max(0.6, base + 0.05), (base, after)
        assert vers == ([60, 60] if mode == "sync" else [120, 120])
        assert servers[0].tables["emb"].step == (60 if mode == "sync" else 120)
    finally:
        for s in servers:
            s.stop()


def test_reference_example_job_runs_verbatim(tmp_path):
    """The reference's example ElasticJob (docs/design/elastic-training-operator.md:31-45) with its
    own command line, ``python -m model_zoo.iris.dnn_estimator``, and image names, under the
    local operator: 2 PS + 2 workers + 1 evaluator train the Iris DNN to high accuracy."""
    spec = tmp_path / "job.yaml"
    spec.write_text(textwrap.dedent("""
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
          env: {EDL_NUM_PS: "2", EDL_SAMPLES: "16000"}
        ---
        apiVersion: elastic.easydl.org/v1alpha1
        kind: JobResource
        metadata:
          name: "elastic-training-resource"
        spec:
          selector:
            name: elastic-deepctr-job
          parameter_server:
            replicas: 2
            resource: {cpu: 1, memory: 1024, gpu: 0}
          worker:
            replicas: 2
            resource: {cpu: 1, memory: 1024, gpu: 0}
          evaluator:
            replicas: 1
            resource: {cpu: 1, memory: 1024, gpu: 0}
        """))
    run = tmp_path / "run"
    out = subprocess.run([sys.executable, "-m", "easydl_amd.cli", "submit", str(spec), "--gpus", "",
                          "--run-dir", str(run), "--timeout", "240"], cwd=ROOT, capture_output=True, text=True,
                         env=dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1"), timeout=300)
    assert out.returncode == 0, (out.stdout + out.stderr)[-4000:]
    ev = [json.loads(l) for f in glob.glob(str(run / "events-*.jsonl")) for l in open(f)]
    names = {e.get("proc") for e in ev}
    assert {"worker0", "worker1"} <= names, sorted(n for n in names if n)
    evals = [e for e in ev if e["kind"] == "eval"]
    assert evals and evals[-1]["acc"] > 0.85, evals[-1:]
