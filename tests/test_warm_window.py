"""Warm-up windows for a standby that arrives while the job trains (VERDICT r4 Next #3: a
warm-up never runs beside a training step).  The standby files a request; the job master turns
it into a runtime plan (``warm_window``) applied by every rank at one committed step; the rank on
that GPU grants it and pauses until the warm-up is done (utils/vram.py, master/main.py,
trainer/elastic.py ``_warm_window``, operator/standby.py)."""
import json
import threading
import time
from types import SimpleNamespace

import torch

from easydl_amd.master.main import JobMaster
from easydl_amd.trainer.elastic import ElasticTrainer
from easydl_amd.utils import vram


class _Events:
    def __init__(self):
        self.got = []

    def emit(self, kind, **kw):
        self.got.append(dict(kw, kind=kind))


def test_master_plans_a_warm_window_once_per_request(tmp_path):
    m = JobMaster("ww", 0, run_dir=str(tmp_path))
    kv = m.kv
    kv.set("plan/runtime/1", json.dumps({"bucket_mb": 64.0, "ckpt_interval": 2}))
    kv.add("plan/version", 1)
    m._grant_warm_windows()
    assert kv.counter("plan/version") == 1                 # no request, no plan
    kv.set("standby/roster", "sb0")
    vram.request_warm_window(kv, "sb0", 1, [3, 0])
    m._next_warm_scan = 0.0
    m._grant_warm_windows()
    assert kv.counter("plan/version") == 2
    doc = kv.get("plan/runtime/2")
    assert doc["warm_window"] == {"standby": "sb0", "id": 1, "gpus": [0, 3]}
    assert doc["bucket_mb"] == 64.0 and doc["ckpt_interval"] == 2   # the other knobs carried over
    m._next_warm_scan = 0.0
    m._grant_warm_windows()
    assert kv.counter("plan/version") == 2                 # the same request is planned once
    vram.request_warm_window(kv, "sb1", 1, [1])           # not on the roster (not parked): ignored
    m._next_warm_scan = 0.0
    m._grant_warm_windows()
    assert kv.counter("plan/version") == 2


def _fake_trainer(kv, gpu):
    # the method only needs these attributes; torch.device("cuda", i) touches no GPU
    return SimpleNamespace(device=torch.device("cuda", gpu), kv=kv, step=7, _warm_windows=set(),
                           events=_Events())


def test_rank_on_the_gpu_grants_and_waits_for_the_warm_up(tmp_path):
    m = JobMaster("ww2", 0, run_dir=str(tmp_path))
    kv = m.kv
    kv.set("standby/roster", "sb0")
    vram.request_warm_window(kv, "sb0", 4, [0])
    ww = {"standby": "sb0", "id": 4, "gpus": [0]}

    def standby():   # grant seen -> warm-up -> warm key
        t_end = time.time() + 10
        while not kv.exists("standby/warm_grant/sb0/gpu0") and time.time() < t_end:
            time.sleep(0.01)
        time.sleep(0.3)
        kv.set("standby/warm/sb0/gpu0", json.dumps({"s": 0.3}))

    th = threading.Thread(target=standby)
    th.start()
    tr = _fake_trainer(kv, 0)
    t0 = time.perf_counter()
    ElasticTrainer._warm_window(tr, ww)
    waited = time.perf_counter() - t0
    th.join()
    ev = [e for e in tr.events.got if e["kind"] == "standby_warm_window"]
    assert len(ev) == 1 and ev[0]["warm"] and ev[0]["step"] == 7 and waited >= 0.3
    ElasticTrainer._warm_window(tr, ww)                    # applied again (epoch entry): no second wait
    assert len([e for e in tr.events.got if e["kind"] == "standby_warm_window"]) == 1

    other = _fake_trainer(kv, 1)                           # a rank on another GPU goes on
    ElasticTrainer._warm_window(other, ww)
    assert not other.events.got and not kv.exists("standby/warm_grant/sb0/gpu1")


def test_stale_window_is_skipped(tmp_path):
    m = JobMaster("ww3", 0, run_dir=str(tmp_path))
    kv = m.kv
    kv.set("standby/roster", "sb0")
    vram.request_warm_window(kv, "sb0", 5, [0])
    tr = _fake_trainer(kv, 0)
    ElasticTrainer._warm_window(tr, {"standby": "sb0", "id": 4, "gpus": [0]})   # superseded request
    kv.set("standby/roster", "")
    ElasticTrainer._warm_window(tr, {"standby": "sb0", "id": 5, "gpus": [0]})   # standby gone
    assert not tr.events.got and not kv.exists("standby/warm_grant/sb0/gpu0")


def test_window_ends_when_the_standby_leaves(tmp_path):
    m = JobMaster("ww4", 0, run_dir=str(tmp_path))
    kv = m.kv
    kv.set("standby/roster", "sb0")
    vram.request_warm_window(kv, "sb0", 1, [0])

    def leave():     # the standby took over a dead worker instead of warming up
        time.sleep(0.3)
        kv.set("standby/roster", "")

    th = threading.Thread(target=leave)
    th.start()
    tr = _fake_trainer(kv, 0)
    t0 = time.perf_counter()
    ElasticTrainer._warm_window(tr, {"standby": "sb0", "id": 1, "gpus": [0]})
    th.join()
    assert time.perf_counter() - t0 < 5
    ev = [e for e in tr.events.got if e["kind"] == "standby_warm_window"]
    assert len(ev) == 1 and not ev[0]["warm"]
