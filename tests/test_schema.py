"""Control-plane wire schemas (easydl_amd/api/schema.py)."""
import json
import subprocess
import sys

from easydl_amd.api.schema import SCHEMAS, document, validate
from easydl_amd.api.spec import ElasticJob, JobResource, Resource, RoleResource, load_yaml_docs

REF_YAML = """
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
  name: elastic-training-resource
spec:
  selector:
    name: elastic-deepctr-job  // Job Name
  parameter_server:
    replicas: 4
    resource: {cpu: 4, memory: 4096, disk: 8192, gpu: 1}
  worker:
    replicas: 4
    resource: {cpu: 4, memory: 4096, disk: 8192, gpu: 1}
  evaluator:
    replicas: 1
    resource: {cpu: 4, memory: 4096, disk: 8192, gpu: 1}
  resource_updation:
    - name: "elastic-deepctr-job-ps-0"
      resource: {cpu: 8, memory: 8192}
"""


def test_reference_crds_validate():
    for d in load_yaml_docs(REF_YAML):
        assert validate(d) == [], d["kind"]


def test_roundtrip_of_our_dataclasses_validates():
    jr = JobResource("r", "j", {"worker": RoleResource(8, Resource(gpu=1, cu=128, hbm_gb=200))})
    assert validate(jr.to_dict()) == []
    assert validate(ElasticJob(name="j", command="python -m x", standby=1).to_dict()) == []


def test_violations_are_reported_with_paths():
    bad = {"kind": "JobResource", "spec": {"selector": {"name": "j"},
                                             "worker": {"replicas": -1, "resource": {"cu": 300, "gpus": 1}}}}
    errs = validate(bad)
    assert any("$.spec.worker.replicas" in e for e in errs)
    assert any("maximum 256" in e for e in errs)
    assert any("unknown field 'gpus'" in e for e in errs)
    assert validate({"kind": "Nope"}) == ["$: unknown message kind 'Nope'"]


def test_cli_schema_and_validate(tmp_path):
    p = tmp_path / "ref.yaml"
    p.write_text(REF_YAML)
    r = subprocess.run([sys.executable, "-m", "easydl_amd.cli", "validate", str(p)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    r = subprocess.run([sys.executable, "-m", "easydl_amd.cli", "schema", "ResourcePlan"], capture_output=True,
                       text=True)
    assert json.loads(r.stdout)["title"] == "ResourcePlan"
    assert set(SCHEMAS) >= {"ElasticJob", "JobResource", "ResourcePlan", "PlanRequest", "PlanResponse"}
    assert document("ElasticJob")["$id"].endswith("/ElasticJob")


def test_cli_logs(tmp_path):
    (tmp_path / "logs").mkdir()
    (tmp_path / "logs" / "j-worker-0.log").write_text("a\nb\nc\n")
    (tmp_path / "events-worker0.jsonl").write_text('{"ts": 1.0, "mono": 1.0, "proc": "w", "kind": "joined"}\n')
    r = subprocess.run([sys.executable, "-m", "easydl_amd.cli", "logs", "--run-dir", str(tmp_path), "--tail", "2",
                        "--events"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert "==> j-worker-0.log <==" in r.stdout and "b\nc" in r.stdout and '"joined"' in r.stdout
