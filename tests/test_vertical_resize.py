"""Vertical resize by replacement, end to end on the CPU tier (reference
docs/design/elastic-training-operator.md:86-101: ``resource_updation`` launches a new
process with the new resource that replaces the named one), driven by the master's plan
loop from LIVE metrics (reference README.md:21-23; VERDICT r4 "Next" #6 and #7).

* A parameter server publishes its live load (utils/kmix.py via ``metrics/<node>``); the
  real Brain plans more CPUs for it while it runs; the operator replaces it; the old PS
  retires (final snapshot, exit 0), the new one restores exactly that version; training
  completes with every data shard done once.
* A data-parallel worker gets a CU plan from the plan loop (a stand-in Brain service over
  HTTP); the operator replaces it; the old worker leaves at a step boundary, the survivor
  goes on, the new worker (CU-masked environment) rejoins and receives the state; the
  committed step count never goes back and both ranks end bit-identical.
"""
import glob
import json
import os
import subprocess
import sys
import textwrap
import threading
from http.server import BaseHTTPRequestHandler, HTTPServer


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _events(run):
    ev = [json.loads(ln) for f in glob.glob(os.path.join(run, "events-*.jsonl")) for ln in open(f)]
    ev.sort(key=lambda e: e["ts"])
    return ev


def _submit(spec_text, tmp_path, timeout=240, env=None):
    spec = tmp_path / "job.yaml"
    spec.write_text(textwrap.dedent(spec_text))
    run = str(tmp_path / "run")
    r = subprocess.run([sys.executable, "-m", "easydl_amd.cli", "submit", str(spec), "--gpus", "", "--run-dir", run,
                        "--timeout", str(timeout)], cwd=ROOT, capture_output=True, text=True, timeout=timeout + 60,
                       env=dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1", **(env or {})))
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    return _events(run)


def test_brain_resizes_a_running_parameter_server_from_its_live_metrics(tmp_path):
    ev = _submit("""
        apiVersion: elastic.easydl.org/v1alpha1
        kind: ElasticJob
        metadata: {name: vrps}
        spec:
          command: "python -m easydl_amd.examples.mnist"
          parameter_server: {image: local}
          worker: {image: local}
          evaluator: {image: local}
          env: {EDL_SAMPLES: "40000", EDL_SHARD: "512", EDL_BATCH: "64", EDL_PLAN_PERIOD_S: "1",
                EDL_BRAIN_PS_BUSY_HIGH: "0.0", EDL_BRAIN_PS_CPU_MAX: "2", EDL_PS_METRICS_S: "0.5"}
        ---
        apiVersion: elastic.easydl.org/v1alpha1
        kind: JobResource
        metadata: {name: vrps-resource}
        spec:
          selector: {name: vrps}
          parameter_server: {replicas: 1, resource: {cpu: 1, memory: 1024, gpu: 0}}
          worker: {replicas: 2, resource: {cpu: 1, memory: 1024, gpu: 0}}
          evaluator: {replicas: 1, resource: {cpu: 1, memory: 1024, gpu: 0}}
        """, tmp_path)
    kinds = [e["kind"] for e in ev]
    replan = next(e for e in ev if e["kind"] == "replan")
    assert "vrps-ps-0" in replan["reason"] and "2 CPUs" in replan["reason"], replan
    replace = [e for e in ev if e["kind"] == "replace"]
    assert len(replace) == 1 and replace[0]["name"] == "vrps-ps-0" and replace[0]["resource"]["cpu"] == 2.0
    spawns = [e for e in ev if e["kind"] == "spawn" and e.get("name") == "vrps-ps-0"]
    assert [s["gen"] for s in spawns] == [0, 1] and spawns[1]["resource"]["cpu"] == 2.0
    old_exit = next(e for e in ev if e["kind"] == "exit" and e.get("pid") == spawns[0]["pid"])
    # the plan came from the running process's own metrics: it was still alive when replanned
    assert old_exit["code"] == 0 and not old_exit["signal"] and old_exit["ts"] > replan["ts"]
    retired = next(e for e in ev if e["kind"] == "ps_retired")
    restored = [e for e in ev if e["kind"] == "ps_restored"]
    assert len(restored) == 1 and restored[0]["version"] == retired["version"] > 0   # no update lost
    assert restored[0]["ts"] > retired["ts"]
    done = [e["shard"] for e in ev if e["kind"] == "shard_done"]
    assert sorted(done) == list(range((40000 + 511) // 512))     # every shard exactly once
    assert "job_complete" in kinds
    assert [e for e in ev if e["kind"] == "eval"][-1]["acc"] > 0.6


class _Brain(BaseHTTPRequestHandler):
    """A Brain service that plans 128 CUs for worker 1 the first time it sees it."""
    issued = []

    def log_message(self, *a):
        pass

    def do_POST(self):
        body = json.loads(self.rfile.read(int(self.headers.get("Content-Length", 0))) or b"{}")
        out = None
        if self.path == "/next_plan":
            nodes = [n for n in body.get("metrics", {}) if n.startswith("vrw-worker-1:")]
            if nodes and not self.issued:
                self.issued.append(nodes[0])
                plan = dict(body["plan"], per_rank={nodes[0]: {"cu": 128}}, reason="test: 128 CUs for worker 1")
                out = plan
        data = json.dumps(out).encode()
        self.send_response(200)
        self.send_header("Content-Length", str(len(data)))
        self.end_headers()
        self.wfile.write(data)


def test_plan_loop_replaces_a_running_worker_with_a_cu_plan(tmp_path):
    _Brain.issued = []
    srv = HTTPServer(("127.0.0.1", 0), _Brain)
    th = threading.Thread(target=srv.serve_forever, daemon=True)
    th.start()
    try:
        ev = _submit("""
            apiVersion: elastic.easydl.org/v1alpha1
            kind: ElasticJob
            metadata: {name: vrw}
            spec:
              command: "python -m easydl_amd.trainer.fault_bench --worker"
              worker: {image: local}
              env: {EDL_BENCH_STEPS: "400", EDL_BENCH_CKPT: "4", EDL_PLANNED_WORKERS: "2", EDL_PLAN_PERIOD_S: "0.5",
                    EDL_BENCH_MBS: "1", EDL_BENCH_ACCUM: "2"}
            ---
            apiVersion: elastic.easydl.org/v1alpha1
            kind: JobResource
            metadata: {name: vrw-resource}
            spec:
              selector: {name: vrw}
              worker: {replicas: 2, resource: {cpu: 1, memory: 1024, gpu: 0}}
            """, tmp_path, env={"EDL_BRAIN_URL": f"http://127.0.0.1:{srv.server_port}"})
    finally:
        srv.shutdown()
    assert len(_Brain.issued) == 1
    replace = [e for e in ev if e["kind"] == "replace"]
    assert len(replace) == 1 and replace[0]["name"] == "vrw-worker-1" and replace[0]["resource"]["cu"] == 128
    spawns = [e for e in ev if e["kind"] == "spawn" and e.get("name") == "vrw-worker-1"]
    assert [s["gen"] for s in spawns] == [0, 1] and spawns[1]["resource"]["cu"] == 128
    old_exit = next(e for e in ev if e["kind"] == "exit" and e.get("pid") == spawns[0]["pid"])
    assert old_exit["code"] == 0 and not old_exit["signal"]        # left at a step boundary, not killed
    # committed steps never go back, whatever the world size
    steps = [e["step"] for e in ev if e["kind"] == "step_done" and e["proc"] == "worker0"]
    assert steps == sorted(steps) and steps[-1] == 400
    finals = [e for e in ev if e["kind"] == "final_state"]
    worlds = [e["world"] for e in ev if e["kind"] == "epoch_formed" and e["ts"] < finals[0]["ts"]]
    assert worlds == [2, 1, 2], worlds            # shrink while replaced, back to 2 (then training ends)
    assert len(finals) == 2 and {f["step"] for f in finals} == {400}
    assert finals[0]["crc"] == finals[1]["crc"]                   # bit-identical ranks
    joined = [e for e in ev if e["kind"] == "state_broadcast"]
    assert joined, "the new worker must receive the state from the survivor"
