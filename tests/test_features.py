"""Job feature extraction (meta-device model analysis) feeding the Brain; shipped tuning files."""
import os

import pytest

from easydl_amd.api.spec import ElasticJob
from easydl_amd.brain.collectors import GpuInfo, NodeInventory
from easydl_amd.brain.planner import JobFeatures, Planner
from easydl_amd.master.features import extract


def test_llama_features_from_env():
    f = extract(ElasticJob(name="j", env={"EDL_MODEL": "llama3-8b", "EDL_SEQ": "8192", "EDL_MBS": "2"}))
    assert 8.0e9 < f["params"] < 8.1e9
    assert f["tokens_per_step_per_rank"] == 16384
    assert abs(f["state_gb_per_rank"] - 128.5) < 1.0          # 16 B/param
    assert 60 < f["activation_gb_per_rank"] < 90


def test_tp_divides_state_and_hints_win():
    f = extract(ElasticJob(name="j", env={"EDL_MODEL": "llama3-70b", "EDL_TP": "8"},
                           features={"activation_gb_per_rank": 50}))
    assert 7.0e10 < f["params"] < 7.1e10 and f["tp"] == 8
    assert f["state_gb_per_rank"] < 145
    assert f["activation_gb_per_rank"] == 50                 # user declaration overrides


def test_unknown_model_is_harmless_and_brain_accepts():
    f = extract(ElasticJob(name="j", features={"model": "my-net", "params": 1e6}))
    assert f["params"] == 1e6
    inv = NodeInventory(gpus=[GpuInfo(i, "gfx950", 256, 288.0) for i in range(8)], cpus=128, host_mem_gb=2048)
    feat = JobFeatures.from_dict(extract(ElasticJob(name="j", env={"EDL_MODEL": "llama3-8b"})))
    plan = Planner().startup_plan(feat, inv)
    assert plan.roles["worker"].replicas == 8
    assert JobFeatures.from_dict(f).params == 1e6


def test_bert_large_ps_plan_is_2ps_6workers_with_cu_hbm():
    """BASELINE config 4: the Brain's startup plan for BERT-large async PS on 8 MI355X."""
    from easydl_amd.api.spec import load_specs
    job, jr = load_specs("examples/bert_ps.yaml")
    assert jr is None and job.mode == "ps"          # no JobResource: the Brain decides
    feat = JobFeatures.from_dict(extract(job))
    assert 3.3e8 < feat.params < 3.5e8
    inv = NodeInventory(gpus=[GpuInfo(i, "gfx950", 256, 288.0) for i in range(8)], cpus=128, host_mem_gb=2048)
    plan = Planner().startup_plan(feat, inv)
    ps, w = plan.roles["parameter_server"], plan.roles["worker"]
    assert (ps.replicas, w.replicas) == (2, 6), plan.reason
    assert ps.resource.gpu == 1 and 0 < ps.resource.cu < 256 and 0 < ps.resource.hbm_gb < 288


def test_gemm_tuning_is_off_without_a_gpu(monkeypatch):
    from easydl_amd.ops import gemm_tuning
    monkeypatch.setenv("EDL_GEMM_TUNING", "use")
    assert gemm_tuning.apply() == "off"          # CPU tier: no TunableOp, no file needed
    assert gemm_tuning.TUNED_FILE.endswith("tunableop_gfx950.csv")


def test_gemm_tuning_select_file_is_curated(monkeypatch):
    """The default mode reads the curated selections: validators of this image plus only
    hipBLASLt entries (each one vetted end to end, profiles/r02_gemm_select_ab.txt)."""
    from easydl_amd.ops import gemm_tuning
    monkeypatch.delenv("EDL_GEMM_TUNING", raising=False)
    assert gemm_tuning.apply() == "off"          # no GPU here
    lines = open(gemm_tuning.SELECT_FILE).read().splitlines()
    vals = {ln.split(",")[1]: ln.split(",")[2] for ln in lines if ln.startswith("Validator,")}
    assert vals["GCN_ARCH_NAME"].startswith("gfx950") and "PT_VERSION" in vals
    entries = [ln.split(",") for ln in lines if not ln.startswith("Validator,")]
    assert entries and all(e[0].startswith("GemmTunableOp_BFloat16") and e[2].startswith("Gemm_Hipblaslt")
                           for e in entries)
    assert any(e[1] == "tn_14336_4096_16384_ld_16384_16384_14336" for e in entries)   # down-proj wgrad


@pytest.mark.gpu
def test_a_stale_shared_tunableop_file_is_not_read():
    """TunableOp reads its output file when it starts.  A file left under the old shared per-user
    name, holding a solution index this hipBLASLt lacks, must not reach a new process's GEMMs
    (scripts/tunableop_scratch_probe.py; before the fix the GEMM failed)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "scripts", "tunableop_scratch_probe.py"), "bogus"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "gemm ok True" in r.stdout, (r.stdout[-2000:], r.stderr[-2000:])


def test_shipped_miopen_find_db_installs_into_a_scratch_copy(monkeypatch, tmp_path):
    import tempfile
    from easydl_amd.ops import conv_tuning
    monkeypatch.delenv("MIOPEN_USER_DB_PATH", raising=False)
    monkeypatch.delenv("EDL_MIOPEN_DB", raising=False)
    monkeypatch.setattr(tempfile, "tempdir", str(tmp_path))
    d = conv_tuning.install()
    assert d is not None and os.environ["MIOPEN_USER_DB_PATH"] == d and d.startswith(str(tmp_path))
    assert any(f.endswith(".ufdb.txt") for f in os.listdir(d))
    monkeypatch.setenv("MIOPEN_USER_DB_PATH", "/elsewhere")            # a user's own db wins
    assert conv_tuning.install() is None and os.environ["MIOPEN_USER_DB_PATH"] == "/elsewhere"
    monkeypatch.delenv("MIOPEN_USER_DB_PATH")
    monkeypatch.setenv("EDL_MIOPEN_DB", "0")
    assert conv_tuning.install() is None and "MIOPEN_USER_DB_PATH" not in os.environ
