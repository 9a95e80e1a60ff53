"""End to end on CPU: `edl submit` -> operator spawns the master first, applies the
JobResource, spawns workers; a worker is killed mid-run, the survivors shrink
and continue, the operator replaces the dead worker, the replacement joins
(scale-up with state broadcast) and the job completes."""
import glob
import json
import os
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.slow
def test_submit_kill_replace_complete(tmp_path):
    spec = tmp_path / "job.yaml"
    spec.write_text(textwrap.dedent(f"""
        apiVersion: edl.mi355x/v1
        kind: ElasticJob
        metadata: {{name: e2e}}
        spec:
          command: "python {ROOT}/tests/helpers/elastic_worker.py"
          min_workers: 1
          max_workers: 3
          env: {{TEST_STEPS: "40", TEST_GB: "6", TEST_STEP_SLEEP: "0.1", EDL_FAULT: "kill@step=6,index=1"}}
        ---
        apiVersion: edl.mi355x/v1
        kind: JobResource
        metadata: {{name: e2e-resource}}
        spec:
          selector: {{name: e2e}}
          worker: {{replicas: 3, resource: {{cpu: 1, gpu: 0}}}}
        """))
    r = subprocess.run([sys.executable, "-m", "easydl_amd.cli", "submit", str(spec), "--gpus", "",
                        "--run-dir", str(tmp_path / "run"), "--timeout", "240"], cwd=ROOT,
                       capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1"))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = [json.load(open(f)) for f in glob.glob(str(tmp_path / "run" / "res*.json"))]
    assert len(res) == 3, res  # workers 0, 2 and the replacement of 1
    assert len({x["hash"] for x in res}) == 1, "replicas diverged"
    assert all(x["step"] == 40 for x in res)
    worlds = max(res, key=lambda x: len(x["worlds"]))["worlds"]
    assert 2 in worlds and worlds[-1] == 3, worlds
    ev = [json.loads(l) for f in glob.glob(str(tmp_path / "run" / "events-operator.jsonl")) for l in open(f)]
    spawns = [e for e in ev if e["kind"] == "spawn"]
    assert spawns[0]["name"] == "e2e-trainer-0"
    assert sum(1 for e in spawns if e["name"] == "e2e-worker-1") == 2


@pytest.mark.slow
def test_hot_standby_takes_over_failed_worker(tmp_path):
    """A parked, pre-imported standby becomes the dead worker (same name, new
    generation) without a new process: the replacement joins faster than a cold spawn."""
    spec = tmp_path / "job.yaml"
    spec.write_text(textwrap.dedent("""
        apiVersion: edl.mi355x/v1
        kind: ElasticJob
        metadata: {name: hot}
        spec:
          command: "python -m tests.helpers.elastic_worker"
          min_workers: 1
          max_workers: 2
          standby: 1
          env: {TEST_STEPS: "40", TEST_GB: "4", TEST_STEP_SLEEP: "0.15", EDL_FAULT: "kill@step=12,index=1"}
        ---
        apiVersion: edl.mi355x/v1
        kind: JobResource
        metadata: {name: hot-resource}
        spec:
          selector: {name: hot}
          worker: {replicas: 2, resource: {cpu: 1, gpu: 0}}
        """))
    run = tmp_path / "run"
    r = subprocess.run([sys.executable, "-m", "easydl_amd.cli", "submit", str(spec), "--gpus", "",
                        "--run-dir", str(run), "--timeout", "240"], cwd=ROOT,
                       capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1"))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    ev = [json.loads(l) for f in glob.glob(str(run / "events-*.jsonl")) for l in open(f)]
    spawns = [e for e in ev if e["kind"] == "spawn" and e.get("name") == "hot-worker-1"]
    assert len(spawns) == 2 and spawns[1].get("standby"), spawns
    sb = [e for e in ev if e["kind"] == "standby_spawn"]
    assert spawns[1]["pid"] in {e["pid"] for e in sb}           # no new process: the standby's pid
    res = [json.load(open(f)) for f in glob.glob(str(run / "res*.json"))]
    assert len({x["hash"] for x in res}) == 1 and all(x["step"] == 40 for x in res), res


@pytest.mark.slow
def test_scale_up_mid_run_through_jobresource():
    """BASELINE config 2 path on CPU: a JobResource update mid-run (what `edl scale` writes)
    grows the world 1 -> 3 without restarting the running worker."""
    r = subprocess.run([sys.executable, "-m", "easydl_amd.trainer.scale_bench", "--start", "1", "--end", "3",
                        "--steps", "300", "--scale-step", "5"], cwd=ROOT, capture_output=True, text=True,
                       timeout=400, env=dict(os.environ, PYTHONPATH=ROOT))
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert r.returncode == 0, r.stderr[-3000:]
    assert set(out["images_per_s_by_world"]) == {"1", "3"}, out
    s = out["scale_up_s"]
    assert s["epoch_formed"] is not None and s["first_step"] is not None and s["first_step"] < 30, s
