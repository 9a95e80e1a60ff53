"""Job master process (the "master face" of EasyDL's ElasticTrainer:
reference docs/design/elastic-training-operator.md:105-112).

Hosts the job's TCPStore server and runs:
* the dynamic-membership :class:`RendezvousManager` (epochs, abort flags);
* the failure detector inputs: exit events written by the operator's
  supervisor under ``ev/exit/<node>`` and heartbeats (``hb/<node>``);
* the plan loop: job features -> Brain startup plan -> JobResource, then
  periodic re-plans from collected metrics — see
  :mod:`easydl_amd.master.planner`.

Run: ``python -m easydl_amd.master.main --job NAME --port P [--min 1 --max 8]``.
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import signal
import threading
import time

from easydl_amd.master.rendezvous import RendezvousConfig, RendezvousManager
from easydl_amd.master.store import KV, make_tcp_store
from easydl_amd.utils.events import EventLog

log = logging.getLogger("edl.master")


class JobMaster:
    def __init__(self, job: str, port: int, host: str = "127.0.0.1", rdzv: RendezvousConfig | None = None,
                 run_dir: str | None = None, planner=None):
        self.job = job
        self.host = host
        self.store = make_tcp_store(host, port, True)
        self.port = self.store.port
        self.kv = KV(self.store, f"edl/{job}")
        self.run_dir = run_dir or os.path.join("runs", job)
        self.events = EventLog(os.path.join(self.run_dir, "events-master.jsonl"), proc="master")
        self.rdzv = RendezvousManager(self.kv, rdzv or RendezvousConfig(), events=self.events)
        self.planner = planner
        self.rdzv.on_dead.append(self._requeue_data)
        self._stop = threading.Event()
        self._threads: list[threading.Thread] = []

    def _requeue_data(self, node: str) -> None:
        cfg = self.kv.get("data/config")
        if not cfg:
            return
        from easydl_amd.master.dispatcher import ShardDispatcher
        d = ShardDispatcher(self.kv, int(cfg["n"]), int(cfg["shard_size"]), int(cfg.get("epochs", 1)))
        shards = d.requeue_dead({node})
        if shards:
            self.events.emit("data_requeued", node=node, shards=shards)

    # exit events from the operator's supervisor -> immediate death marks
    def _scan_exit_events(self):
        for n in self.rdzv.joined():
            if self.kv.exists(f"ev/exit/{n}") and not self.kv.exists(f"ev/dead/{n}"):
                info = self.kv.get(f"ev/exit/{n}")
                self.rdzv.mark_dead(n, f"process exit {info}")

    def _grant_warm_windows(self) -> None:
        """A parked standby's request for a warm-up window (utils/vram.py) becomes a runtime plan
        with a ``warm_window``: every rank applies it at one committed step, the ranks on its
        GPUs pause for the warm-up, and no warm-up GEMM runs beside a training step."""
        now = time.monotonic()
        if now < getattr(self, "_next_warm_scan", 0.0):
            return
        self._next_warm_scan = now + 0.5
        from easydl_amd.utils import vram
        done = self.__dict__.setdefault("_warm_granted", set())
        for name in vram.roster(self.kv):
            req = vram.read_warm_request(self.kv, name)
            if not req or (name, req["id"]) in done:
                continue
            done.add((name, req["id"]))
            cur = self.kv.counter("plan/version")
            doc = self.kv.get(f"plan/runtime/{cur}") if cur else None
            doc = dict(doc) if isinstance(doc, dict) else {}
            doc["warm_window"] = {"standby": name, "id": req["id"], "gpus": req["gpus"]}
            self.kv.set(f"plan/runtime/{cur + 1}", json.dumps(doc))
            self.kv.add("plan/version", 1)
            self.events.emit("warm_window_planned", standby=name, id=req["id"], gpus=req["gpus"], version=cur + 1)

    def _loop(self, period):
        while not self._stop.is_set():
            try:
                self._scan_exit_events()
                self.rdzv.tick()
                self._grant_warm_windows()
                if self.planner is not None:
                    self.planner.maybe_replan(self)
            except Exception as e:
                log.warning("master tick failed: %s", e)
            self._stop.wait(period)

    def start(self, period: float = 0.01) -> "JobMaster":
        t = threading.Thread(target=self._loop, args=(period,), name="edl-master", daemon=True)
        t.start()
        self._threads.append(t)
        self.kv.set("master/info", json.dumps({"host": self.host, "port": self.port, "pid": os.getpid(),
                                               "ts": time.time()}))
        self.events.emit("master_started", port=self.port)
        return self

    def serve_metrics(self, port: int = 0) -> int:
        """Prometheus text endpoint: per-member training metrics reported to the store."""
        from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

        from easydl_amd.utils.metrics import render_prometheus
        master = self

        class H(BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def do_GET(self):
                ms = {n: m for n in master.rdzv.members() if (m := master.kv.get(f"metrics/{n}"))}
                body = render_prometheus(ms, master.job).encode()
                self.send_response(200)
                self.send_header("Content-Type", "text/plain; version=0.0.4")
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

        srv = ThreadingHTTPServer(("127.0.0.1", port), H)
        threading.Thread(target=srv.serve_forever, daemon=True, name="edl-metrics").start()
        self._metrics_srv = srv
        return srv.server_address[1]

    def stop(self):
        self._stop.set()
        for t in self._threads:
            t.join(timeout=2)

    def serve_forever(self):
        try:
            while not self._stop.wait(0.5):
                if self.kv.exists("master/shutdown"):
                    break
        finally:
            self.stop()


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--job", default=os.environ.get("EDL_JOB", "job"))
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=int(os.environ.get("EDL_MASTER_PORT", 29400)))
    ap.add_argument("--min", type=int, default=1)
    ap.add_argument("--max", type=int, default=8)
    ap.add_argument("--initial", type=int, default=0, help="first epoch waits for this many workers")
    ap.add_argument("--join-window", type=float, default=0.5)
    ap.add_argument("--hb-timeout", type=float, default=15.0)
    ap.add_argument("--policy", default="shrink")
    ap.add_argument("--granule", type=int, default=int(os.environ.get("EDL_TP", 1)),
                    help="world sizes are multiples of this (tensor-parallel degree)")
    ap.add_argument("--run-dir", default=os.environ.get("EDL_RUN_DIR"))
    ap.add_argument("--job-spec", default=None, help="ElasticJob JSON/YAML: enables the Brain plan loop")
    ap.add_argument("--brain-url", default=os.environ.get("EDL_BRAIN_URL"))
    ap.add_argument("--plan-period", type=float, default=float(os.environ.get("EDL_PLAN_PERIOD_S", 30.0)))
    ap.add_argument("--job-resource", default=None, help="user JobResource JSON/YAML (Brain not consulted)")
    ap.add_argument("--metrics-port", type=int, default=-1, help="Prometheus endpoint port (0 = any, -1 = off)")
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s [master] %(message)s")
    cfg = RendezvousConfig(min_nodes=a.min, max_nodes=a.max, initial_nodes=a.initial, join_window_s=a.join_window,
                           granule=a.granule,
                           heartbeat_timeout_s=a.hb_timeout, policy=a.policy)
    planner = None
    if a.job_spec:
        from easydl_amd.api.spec import ElasticJob, load_yaml_docs
        from easydl_amd.brain.service import BrainClient
        from easydl_amd.master.planner import PlanLoop
        txt = open(a.job_spec).read()
        doc = json.loads(txt) if txt.lstrip().startswith("{") else load_yaml_docs(txt)[0]
        planner = PlanLoop(ElasticJob.from_dict(doc), BrainClient(a.brain_url), period_s=a.plan_period)
    m = JobMaster(a.job, a.port, a.host, cfg, a.run_dir, planner=planner)
    if a.job_resource:
        from easydl_amd.api.spec import JobResource, load_yaml_docs
        txt = open(a.job_resource).read()
        doc = json.loads(txt) if txt.lstrip().startswith("{") else load_yaml_docs(txt)[0]
        m.kv.set("jobresource", json.dumps(JobResource.from_dict(doc).to_dict()))
    m.start()
    if a.metrics_port >= 0:
        m.events.emit("metrics_endpoint", port=m.serve_metrics(a.metrics_port))
    signal.signal(signal.SIGTERM, lambda *_: m._stop.set())
    print(json.dumps({"master_port": m.port}), flush=True)
    m.serve_forever()


if __name__ == "__main__":
    main()
