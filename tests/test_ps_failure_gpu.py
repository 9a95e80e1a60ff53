"""VERDICT r5 Next #8: a GPU parameter server dies while its workers have its shard IPC-mapped.

Config-4 layout on one GPU (BERT, async PS, GPU transport: pushes and pulls through IPC-mapped
HBM, pipelined pushes), run through the local operator: PS 0 SIGKILLs itself in the middle of
the traffic (``kill@step=<update>,role=ps``).  The operator replaces it; the replacement restores
the newest GPU-shard snapshot from /dev/shm; each worker's push that was in flight to the dead
PS is counted lost (its gradients were in the dead PS's inbox), the worker maps the replacement's
buffers and goes on.  The replacement continues the version count from the highest version a
worker saw, so no worker ever observes a version going back.  Every data shard is trained
exactly once.  The PS time-to-recover (kill -> first update applied by the replacement) and the
lost pushes / updates are printed (profiles/r06_ps_failure_gpu.md)."""
import glob
import json
import os
import subprocess
import sys
import textwrap

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_gpu_ps_killed_under_ipc_traffic_is_replaced_and_training_continues(tmp_path):
    samples, shard = 24000, 480
    spec = tmp_path / "job.yaml"
    spec.write_text(textwrap.dedent(f"""
        apiVersion: elastic.easydl.org/v1alpha1
        kind: ElasticJob
        metadata: {{name: psfail}}
        spec:
          command: "python -m easydl_amd.examples.bert_ps"
          parameter_server: {{image: local}}
          worker: {{image: local}}
          env: {{EDL_MODEL: bert-tiny, EDL_SEQ: "64", EDL_BATCH: "16", EDL_SAMPLES: "{samples}",
                EDL_SHARD: "{shard}", EDL_PS_TRANSPORT: ipc, EDL_PS_PIPELINE: "1",
                EDL_PS_SNAPSHOT_EVERY: "25", EDL_PS_SNAPSHOT_S: "0.2",
                EDL_FAULT: "kill@step=300,role=ps,index=0"}}
        ---
        apiVersion: elastic.easydl.org/v1alpha1
        kind: JobResource
        metadata: {{name: psfail-resource}}
        spec:
          selector: {{name: psfail}}
          parameter_server: {{replicas: 1, resource: {{cpu: 2, memory: 4096, gpu: 1}}}}
          worker: {{replicas: 2, resource: {{cpu: 2, memory: 4096, gpu: 1}}}}
        """))
    run = tmp_path / "run"
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    r = subprocess.run([sys.executable, "-m", "easydl_amd.cli", "submit", str(spec), "--gpus", "0,0,0",
                        "--run-dir", str(run), "--timeout", "200"], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=260)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    ev = sorted((json.loads(ln) for f in glob.glob(str(run / "events-*.jsonl")) for ln in open(f)),
                key=lambda e: e["ts"])
    fault = next(e for e in ev if e["kind"] == "fault_injected")
    assert fault["proc"] == "ps0"
    restored = [e for e in ev if e["kind"] == "ps_restored" and e.get("gen", 0) >= 1]
    assert restored, "the replacement PS did not restore the shard snapshot"
    first = next(e for e in ev if e["kind"] == "ps_first_update" and e["ts"] > fault["ts"])
    reconnects = [e for e in ev if e["kind"] == "ps_reconnected"]
    assert reconnects, "no worker re-mapped the replacement PS"
    assert not [e for e in ev if e["kind"] == "ps_version_went_back"]
    done = [e for e in ev if e["kind"] == "worker_done"]
    assert len(done) == 2 and all(d["transport"] == "ipc" for d in done), done
    shards = {e["shard"] for e in ev if e["kind"] == "shard_done"}
    assert shards == set(range((samples + shard - 1) // shard)), sorted(shards)
    adopted = [e for e in ev if e["kind"] == "ps_version_adopted"]
    ttr = first["ts"] - fault["ts"]
    summary = {
        "ps_ttr_s": round(ttr, 3), "killed_at_version": fault["step"],
        "restored_version": restored[0]["version"], "restore_s": restored[0].get("s"),
        "version_adopted": adopted[-1]["version"] if adopted else None,
        "lost_updates": adopted[-1].get("lost_updates") if adopted else 0,
        "lost_pushes": sum(e["lost"] for e in reconnects),
        "worker_remap_s": [e["s"] for e in reconnects],
        "final_versions": [d["versions"] for d in done], "worker_steps": [d["steps"] for d in done],
        "respawn_s": round(next(e["ts"] for e in ev if e["kind"] == "spawn" and e.get("role") == "parameter_server"
                                and e["ts"] > fault["ts"]) - fault["ts"], 3),
    }
    print("\n[ps-failure-gpu]", json.dumps(summary))
    assert ttr < 60, summary
    assert summary["lost_pushes"] <= 4, summary
    assert all(v[0] >= fault["step"] for v in summary["final_versions"]), summary
