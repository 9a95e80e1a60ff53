"""Parameter-server mode roles: PS, worker, evaluator.

Launched by the local ElasticOperator with the ``EDL_*`` environment; one
entry point (e.g. ``python -m easydl_amd.examples.mnist``) dispatches on
``EDL_ROLE``.  Workers pull the latest parameters from every PS shard, run
forward/backward on a data shard claimed from the master's dispatcher and push
gradients; PS shards apply them (async, or sync rounds over the live workers).
The evaluator periodically pulls and scores the model (reference
docs/design/elastic-training-operator.md:43-44,79-85).
"""
from __future__ import annotations

import json
import logging
import os
import time

import torch

from easydl_amd.master.dispatcher import ShardDispatcher
from easydl_amd.master.rendezvous import RendezvousClient
from easydl_amd.master.store import KV, make_tcp_store
from easydl_amd.ps.client import PSClient, shard_of, store_resolver
from easydl_amd.ps.embedding import table_shard_spec
from easydl_amd.ps.server import ParameterServer, PSSnapshotter
from easydl_amd.trainer.context import TrainerContext
from easydl_amd.utils import fault
from easydl_amd.utils.events import EventLog

log = logging.getLogger("edl.ps_trainer")


def _kv(ctx: TrainerContext) -> KV:
    return KV(make_tcp_store(ctx.master_addr, ctx.master_port, False), f"edl/{ctx.job}")


def _world(kv) -> int:
    e = kv.counter("rdzv/epoch")
    a = kv.get(f"rdzv/assign/{e}") if e else None
    return int(a["world"]) if a else 1


def run_ps(model_fn, num_ps: int, ctx: TrainerContext | None = None, *, optimizer="adam", lr=1e-3, mode="async",
           snapshot_every: int | None = None, device="cpu", seed: int = 1234, sparse_optimizer: str | None = None,
           sparse_lr: float | None = None) -> None:
    """``snapshot_every``: updates between in-memory snapshots of the shard (EDL_PS_SNAPSHOT_EVERY,
    default 20; 0 = none), and for a GPU shard at least EDL_PS_SNAPSHOT_S seconds apart (default
    5).  Each snapshot copies the whole shard state to host DRAM, which a PS sharing its GPU pays
    in copy kernels beside the workers: every 20 updates cost BERT-large 28 % of a per-GPU
    layout's throughput (profiles/r05_ps_per_gpu.md).  Async SGD loses at most those seconds of
    updates on a PS failure."""
    if snapshot_every is None:
        snapshot_every = int(os.environ.get("EDL_PS_SNAPSHOT_EVERY", 20))
    snapshot_min_s = float(os.environ.get("EDL_PS_SNAPSHOT_S", 5.0 if torch.device(device).type == "cuda" else 0))
    ctx = ctx or TrainerContext.from_env()
    kv = _kv(ctx)
    events = EventLog(os.path.join(ctx.run_dir, f"events-ps{ctx.index}.jsonl"), proc=f"ps{ctx.index}")
    gen = int(os.environ.get("EDL_GENERATION", 0))
    torch.manual_seed(seed)
    model = model_fn(device)
    snap = PSSnapshotter(ctx.job, ctx.index)
    ps = ParameterServer(ctx.index, shard_of(model, num_ps, ctx.index), optimizer=optimizer, lr=lr, mode=mode,
                         expected_workers=lambda: _world(kv), device=device, snapshot=snap,
                         snapshot_every=snapshot_every, snapshot_min_s=snapshot_min_s,
                         tables=table_shard_spec(model, num_ps, ctx.index),
                         sparse_optimizer=sparse_optimizer, sparse_lr=sparse_lr, seed=seed)
    del model  # the PS keeps only its shard
    ps.events = events
    handoff = _await_predecessor(kv, ctx.index, gen, events)
    t_restore = time.perf_counter()
    if snap.restore(ps):
        events.emit("ps_restored", version=ps.version, handoff=handoff, gen=gen,
                    s=round(time.perf_counter() - t_restore, 3))
    inj = fault.FaultInjector.from_env(ctx, events)
    first = {"done": gen == 0}

    def on_apply(p):
        # a PS fault fires at an update count (``kill@step=<version>,role=ps``): mid-traffic,
        # with workers' pushes in flight; a replacement marks its first applied update (PS TTR)
        if not first["done"]:
            first["done"] = True
            events.emit("ps_first_update", version=p.version, gen=gen)
        inj.maybe_inject("step_start", p.version)
    ps.on_apply = on_apply
    if snapshot_every > 0:
        snap.prepare(ps)
    ps.start()
    kv.set(f"ps/addr/{ctx.index}", json.dumps({"host": ps.host, "port": ps.port, "pid": os.getpid(), "gen": gen}))
    events.emit("ps_started", port=ps.port, params=ps.state.numel, gen=gen)
    from easydl_amd.utils.metrics import cu_count, publish_role_metrics
    t_start, next_pub = time.time(), 0.0
    try:
        while not kv.exists("job/done") and not ps._stop.is_set():
            if kv.exists(f"rdzv/leave/{ctx.node_id}"):
                # replaced (resource_updation) or scaled down: hand the shard over, then exit 0
                t0 = time.perf_counter()
                ver = ps.retire()
                kv.delete(f"metrics/{ctx.node_id}")
                kv.set(f"ps/handoff/{ctx.index}", json.dumps({"gen": gen, "version": ver, "pid": os.getpid()}))
                events.emit("ps_retired", version=ver, s=round(time.perf_counter() - t0, 3), gen=gen)
                return
            if time.time() >= next_pub:
                # live metrics for the Brain: this rank is no rendezvous member, so it registers itself
                mix = ps.kmix.snapshot()
                up = max(1e-3, min(time.time() - t_start, ps.kmix.window_s))
                publish_role_metrics(kv, ctx.node_id, {
                    "role": "ps", "step": ps.version, "ts": time.time(), "gpu_mix": mix,
                    "busy_frac": round(mix["gpu_s"] / up, 4) if mix else 0.0, "device": ps.state.device.type,
                    "cu": cu_count(ctx.cu_mask), "cpu": int(os.environ.get("OMP_NUM_THREADS", 0) or 0)})
                next_pub = time.time() + float(os.environ.get("EDL_PS_METRICS_S", 2.0))
            time.sleep(0.2)
    finally:
        ps.stop()


def _await_predecessor(kv, index: int, gen: int, events, timeout_s: float = 120.0) -> dict | None:
    """A PS replacing a LIVE predecessor (vertical resize) restores only once that one has
    retired and committed its final snapshot (``ps/handoff/<index>``); a dead predecessor's
    newest snapshot is all there is (the crash path)."""
    prev = kv.get(f"ps/addr/{index}")
    if not prev or int(prev.get("gen", -1)) >= gen or not _alive(prev.get("pid")):
        return None
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < timeout_s:
        h = kv.get(f"ps/handoff/{index}")
        if h and int(h.get("gen", -1)) == int(prev.get("gen", -1)):
            events.emit("ps_handoff_received", version=h.get("version"), wait_s=round(time.perf_counter() - t0, 3))
            return h
        if not _alive(prev.get("pid")):
            break
        time.sleep(0.05)
    events.emit("ps_handoff_missing", predecessor=prev.get("pid"), wait_s=round(time.perf_counter() - t0, 3))
    return None


def _alive(pid) -> bool:
    try:
        os.kill(int(pid), 0)
    except (ProcessLookupError, TypeError, ValueError):
        return False
    except PermissionError:
        return True
    from easydl_amd.utils.procfs import mm_released
    return not mm_released(int(pid))


def _transport(device) -> str:
    """EDL_PS_TRANSPORT (tcp | ipc); ipc needs the worker and the PS shards on GPUs of this node."""
    t = os.environ.get("EDL_PS_TRANSPORT", "tcp")
    return t if torch.device(device).type == "cuda" else "tcp"


class PSWorker:
    def __init__(self, model_fn, num_ps: int, ctx: TrainerContext | None = None, device="cpu", seed: int = 1234,
                 pipeline: bool | None = None):
        """``pipeline`` (async PS only; EDL_PS_PIPELINE): with the GPU transport and a dense
        model, each step's push is sent without waiting for its answer and the next step
        starts from the shard's current parameters (bounded staleness: at most 2 updates
        behind, usually 1), so the PS update runs under the worker's next step
        (PSClient.push_async)."""
        self.ctx = ctx or TrainerContext.from_env()
        self.device = torch.device(device)
        torch.manual_seed(seed)
        self.model = model_fn(self.device)
        self.kv = _kv(self.ctx)
        self.events = EventLog(os.path.join(self.ctx.run_dir, f"events-worker{self.ctx.index}.jsonl"),
                               proc=f"worker{self.ctx.index}")
        self.rdzv = RendezvousClient(self.kv, self.ctx.node_id, {"index": self.ctx.index, "role": "worker"})
        self.client = PSClient(num_ps, store_resolver(self.kv), self.ctx.node_id, transport=_transport(self.device))
        self._phase_sync = os.environ.get("EDL_PS_PHASE_SYNC", "0") == "1"
        self.client.bind(self.model)
        self.fault = fault.FaultInjector.from_env(self.ctx, self.events)
        self.steps = 0
        self._phase = [0.0, 0.0, 0.0]
        if pipeline is None:
            pipeline = os.environ.get("EDL_PS_PIPELINE", "0") == "1"
        self.pipeline = bool(pipeline) and self.client.pipelined()
        self._reconnects_seen = 0
        self._max_versions = [0] * num_ps

    def _watch_versions(self) -> None:
        """PS failures seen by this worker: each reconnect to a replacement PS (with the push it
        lost) becomes an event, and a shard version lower than one already seen is flagged --
        a replacement continues the count from the highest version its workers report."""
        rc = self.client.reconnects
        while self._reconnects_seen < len(rc):
            self.events.emit("ps_reconnected", step=self.steps, **rc[self._reconnects_seen])
            self._reconnects_seen += 1
        for i, v in enumerate(self.client.versions):
            if v < self._max_versions[i]:
                self.events.emit("ps_version_went_back", ps=i, version=v, seen=self._max_versions[i])
            self._max_versions[i] = max(self._max_versions[i], v)

    def fit(self, loss_fn, data, batch_size: int, shard_size: int, epochs: int = 1, on_step=None):
        self.rdzv.join()
        disp = ShardDispatcher(self.kv, len(data), shard_size, epochs)
        self.kv.set("data/config", json.dumps({"n": len(data), "shard_size": shard_size, "epochs": epochs}))
        # GPU transport: the push of step k and the pull for step k+1 share one control
        # message per PS (the PS answers once it has applied the push); the first step pulls
        fused = self.client.transport == "ipc"
        need_pull = True
        try:
            while True:
                shard = disp.claim(self.ctx.node_id)
                if shard is None:
                    break
                lo, hi = disp.shard_range(shard)
                for b0 in range(lo, hi, batch_size):
                    self.fault.maybe_inject("step_start", self.steps, trainer=None)
                    t0 = time.perf_counter()
                    if need_pull:
                        self.client.pull(self.model)
                        need_pull = False
                    elif self.pipeline:
                        self.client.pull_local(self.model)
                    t1 = time.perf_counter()
                    self.model.zero_grad(set_to_none=False)
                    loss = loss_fn(self.model, data.batch(range(b0, min(hi, b0 + batch_size)), self.device))
                    loss.backward()
                    if self._phase_sync and self.device.type == "cuda":
                        # diagnostics only (EDL_PS_PHASE_SYNC=1): exact compute-vs-push split; the GPU
                        # transport otherwise never synchronises the stream on the main thread
                        torch.cuda.current_stream(self.device).synchronize()
                    t2 = time.perf_counter()
                    if self.pipeline:
                        self.client.push_async(self.model, self.steps)
                    else:
                        self.client.push(self.model, self.steps, then_pull=fused)
                        need_pull = not fused
                    t3 = time.perf_counter()
                    self._watch_versions()
                    self.steps += 1
                    self._phase = [a + b for a, b in zip(self._phase, (t1 - t0, t2 - t1, t3 - t2))]
                    if self.steps % 16 == 0:  # where a PS step's time goes (pull / compute / push)
                        self.events.emit("ps_step_phases", steps=16, pull_s=round(self._phase[0] / 16, 4),
                                         compute_s=round(self._phase[1] / 16, 4),
                                         push_s=round(self._phase[2] / 16, 4), transport=self.client.transport)
                        self._phase = [0.0, 0.0, 0.0]
                    if on_step is not None:
                        on_step(self, loss)
                if self.pipeline:
                    self.client.drain()   # a shard is done once its last push is answered
                disp.complete(shard)
                self.events.emit("shard_done", shard=shard, steps=self.steps)
                if self.kv.exists(f"rdzv/leave/{self.ctx.node_id}"):
                    # replaced or scaled down: leave between shards (none half-done, none repeated)
                    self.events.emit("worker_left", steps=self.steps)
                    break
        finally:
            if self.pipeline:
                try:
                    self.client.drain()
                except Exception as e:  # noqa: BLE001 - leaving anyway; the PS side logs it
                    log.warning("last pipelined push not answered: %s", e)
            self.rdzv.leave()
            self.rdzv.stop_heartbeat()
        if disp.done() >= disp.total:
            self.kv.set("job/data_exhausted", "1")
        return self


def run_evaluator(model_fn, num_ps: int, eval_fn, ctx: TrainerContext | None = None, interval_s: float = 1.0,
                  device="cpu", seed: int = 1234):
    ctx = ctx or TrainerContext.from_env()
    kv = _kv(ctx)
    torch.manual_seed(seed)
    model = model_fn(device)
    client = PSClient(num_ps, store_resolver(kv), ctx.node_id, transport=_transport(device))
    client.bind(model)
    events = EventLog(os.path.join(ctx.run_dir, f"events-evaluator{ctx.index}.jsonl"), proc="evaluator")
    last = None
    while not kv.exists("job/done"):
        vers = client.pull(model)
        if vers != last:
            metrics = eval_fn(model)
            metrics["versions"] = vers
            kv.set("eval/latest", json.dumps(metrics))
            events.emit("eval", **metrics)
            last = vers
        if kv.exists("job/data_exhausted"):
            break
        time.sleep(interval_s)
    client.close()
