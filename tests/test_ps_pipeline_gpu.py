"""Pipelined async pushes (PSClient.push_async / PSWorker(pipeline=True)) on the GPU transport:
one PS + one BERT-tiny worker on GPU 0 through the local operator.  Every push is applied
(the shard's version equals the worker's step count), and the MLM loss goes down with the
worker training on parameters at most two updates old."""
import glob
import json
import os
import subprocess
import sys

import pytest
import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
@pytest.mark.parametrize("pipeline", ["1", "0"])
def test_bert_ps_pipelined_pushes_all_applied(tmp_path, pipeline):
    from easydl_amd.api.spec import JobResource, Resource, RoleResource, load_specs
    job, _ = load_specs(os.path.join(ROOT, "examples", "bert_ps.yaml"))
    steps, b = 64, 8
    job.env.update({"EDL_MODEL": "bert-tiny", "EDL_SEQ": "64", "EDL_BATCH": str(b), "EDL_SAMPLES": str(steps * b),
                    "EDL_SHARD": str(8 * b), "EDL_PS_PIPELINE": pipeline})
    jr = JobResource(f"{job.name}-resource", job.name, {
        "parameter_server": RoleResource(1, Resource(gpu=1, cpu=2)),
        "worker": RoleResource(1, Resource(gpu=1, cpu=2))})
    spec = tmp_path / "job.yaml"
    spec.write_text(yaml.safe_dump_all([job.to_dict(), jr.to_dict()]))
    run = tmp_path / "run"
    r = subprocess.run([sys.executable, "-m", "easydl_amd.cli", "submit", str(spec), "--gpus", "0,0",
                        "--run-dir", str(run), "--timeout", "240"], cwd=ROOT, capture_output=True, text=True,
                       timeout=300)
    logs = "".join(open(f, errors="replace").read()[-2000:] for f in glob.glob(str(run / "logs" / "*.log")))
    assert r.returncode == 0, r.stderr[-2000:] + logs
    done = [json.loads(ln) for f in glob.glob(str(run / "events-worker*.jsonl")) for ln in open(f)
            if '"worker_done"' in ln]
    assert len(done) == 1, logs
    d = done[0]
    assert d["transport"] == "ipc" and d["pipeline"] == (pipeline == "1"), d
    assert d["steps"] == steps and d["versions"] == [steps], d      # every push applied exactly once
    assert d["last_loss"] < d["first_loss"], d
