"""ElasticTrainer — the library face of EasyDL's ElasticTrainer (reference
README.md:11, "a framework to use EasyDL in training"), all-reduce mode.

A user gives a model factory, a loss function and a data source; the trainer
owns the loop so that membership changes and failures are handled *inside*
the job without restarting processes:

* join the job master's rendezvous, wait for an epoch assignment, build the
  epoch's communicators (RCCL data plane + gloo control plane);
* run each step: micro-batches (global batch preserved across world sizes),
  backward with bucketed all-reduce overlapped (ElasticDDP), host sync point;
* agree on the step through the store-coordinated commit (apply or drop on
  EVERY rank), then run the fused clip + AdamW;
* a watchdog thread aborts the communicator the moment the master flags the
  epoch as broken (dead/hung peer), so no rank stays stuck in a collective;
* on a new epoch: rebuild communicators, agree on the newest committed state
  and broadcast it to joiners (survivors are already identical), re-shard
  data, continue.  Time-to-recover phases are logged as events.

Usage::

    trainer = ElasticTrainer(lambda dev: Llama(cfg, device=dev), global_batch=64, micro_batch=1)
    trainer.fit(lambda model, batch: model(*batch), SyntheticTokens(cfg.vocab_size, 8192), num_steps=1000)
"""
from __future__ import annotations

import logging
import os
import threading
import time

import torch
import torch.distributed as dist

from easydl_amd.master.rendezvous import RendezvousClient, RendezvousConfig, RendezvousManager
from easydl_amd.master.store import KV, make_tcp_store
from easydl_amd.optim import FlatAdamW, FlatSGD, LRSchedule
from easydl_amd.parallel.comm import CommAborted, Communicator, LocalCommunicator
from easydl_amd.parallel.ddp import ElasticDDP
from easydl_amd.parallel.flat import FlatParams
from easydl_amd.trainer.context import TrainerContext
from easydl_amd.trainer.data import ElasticBatchPlan
from easydl_amd.utils import fault, trace
from easydl_amd.utils.events import EventLog
from easydl_amd.utils.metrics import MetricsReporter
from easydl_amd.utils.resources import apply_plan

log = logging.getLogger(__name__)

# Our watchdog decides when to abort RCCL; the PG must not crash the process itself.
os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "0")


class ElasticTrainer:
    def __init__(self, model_fn, *, optimizer: str = "adamw", lr: float = 3e-4, weight_decay: float = 0.1,
                 betas=(0.9, 0.95), momentum: float = 0.9, max_grad_norm: float = 1.0, global_batch: int | None = None,
                 micro_batch: int = 1, device=None, dtype=torch.bfloat16, bucket_mb: float | None = None,
                 grad_dtype=None, ctx: TrainerContext | None = None, seed: int = 1234, schedule: LRSchedule | None = None,
                 rdzv_config: RendezvousConfig | None = None, checkpoint=None, log_every: int = 0,
                 store=None):
        self.ctx = ctx or TrainerContext.from_env()
        if device is None:
            if torch.cuda.is_available():
                device = torch.device("cuda", self.ctx.gpu or 0)
            else:
                device = torch.device("cpu")
        self.device = torch.device(device)
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
        self.resources = apply_plan(self.ctx, self.device)  # Brain CU mask / HBM cap
        self.events = EventLog(os.path.join(self.ctx.run_dir, f"events-{self.ctx.role}{self.ctx.index}.jsonl"),
                               proc=f"{self.ctx.role}{self.ctx.index}")
        torch.manual_seed(seed)
        self.model = model_fn(self.device)
        self.flat = FlatParams(self.model, weight_decay=weight_decay, grad_dtype=grad_dtype)
        if optimizer == "adamw":
            self.opt = FlatAdamW(self.flat, lr=lr, betas=betas, weight_decay=weight_decay,
                                 max_grad_norm=max_grad_norm, schedule=schedule)
        elif optimizer == "sgd":
            self.opt = FlatSGD(self.flat, lr=lr, momentum=momentum, weight_decay=weight_decay,
                               max_grad_norm=max_grad_norm, schedule=schedule)
        else:
            raise ValueError(f"unknown optimizer {optimizer}")
        self.ddp = ElasticDDP(self.flat, None, bucket_mb=bucket_mb)
        self.global_batch = global_batch
        self.micro_batch = micro_batch
        self.step = 0                # committed optimizer steps
        self.needs_state = True      # fresh process: must receive state unless everyone is fresh
        self.comm = None
        self.assignment = None
        self.checkpoint = checkpoint
        self.log_every = log_every
        self.rdzv_config = rdzv_config
        self._store = store
        self._manager = None
        self._watchdog = None
        self._stop = threading.Event()
        self.fault = fault.FaultInjector.from_env(self.ctx, self.events)
        self.history: list[dict] = []
        self.last_loss = None
        self.tokens_per_sample = 0
        self.metrics = MetricsReporter(path=os.path.join(self.ctx.run_dir, f"metrics-{self.ctx.role}{self.ctx.index}.jsonl"))
        self.plan_version = 0

    # ------------------------------------------------------------------ setup
    def _connect(self):
        if self.ctx.standalone:
            self.kv = None
            self.rdzv = None
            return
        if self._store is None:
            agent = os.environ.get("TORCHELASTIC_USE_AGENT_STORE", "") in ("True", "true", "1")
            is_server = self.ctx.embedded_master and self.ctx.index == 0 and not agent
            self._store = make_tcp_store(self.ctx.master_addr, self.ctx.master_port, is_server)
        self.kv = KV(self._store, f"edl/{self.ctx.job}")
        if self.ctx.embedded_master and self.ctx.index == 0:
            cfg = self.rdzv_config or RendezvousConfig(min_nodes=self.ctx.static_world,
                                                       max_nodes=self.ctx.static_world)
            self._manager = RendezvousManager(self.kv, cfg, events=self.events)
            self._manager.start()
        info = {"index": self.ctx.index, "role": self.ctx.role, "gpu": self.ctx.gpu}
        self.rdzv = RendezvousClient(self.kv, self.ctx.node_id, info)
        self.metrics.kv, self.metrics.node = self.kv, self.ctx.node_id
        self.rdzv.join()
        self.events.emit("joined", node=self.ctx.node_id)

    def _start_watchdog(self):
        def loop():
            while not self._stop.wait(0.01):
                c = self.comm
                if c is None or c.aborted or self.rdzv is None:
                    continue
                try:
                    if self.rdzv.aborted(c.epoch):
                        self.events.emit("abort_seen", epoch=c.epoch)
                        c.abort()
                except Exception:
                    pass

        self._watchdog = threading.Thread(target=loop, name="edl-watchdog", daemon=True)
        self._watchdog.start()

    def _enter_epoch(self):
        """Join the next live epoch; retries when the epoch breaks while it is being built."""
        while True:
            t0 = time.time()
            if self.rdzv is None:
                self.comm = LocalCommunicator(self.device)
                self.assignment = None
            else:
                a = self.rdzv.wait_assignment(after_epoch=self.assignment.epoch if self.assignment else 0)
                self.assignment = a
                self.events.emit("epoch_joined", epoch=a.epoch, rank=a.rank, world=a.world, reason=a.reason)
                if a.world == 1:
                    self.comm = LocalCommunicator(self.device, epoch=a.epoch)
                else:
                    comm = self._build_comm(a)
                    if comm is None:
                        self.events.emit("epoch_skipped", epoch=a.epoch)
                        continue
                    self.comm = comm
            self.events.emit("comm_ready", epoch=self.comm.epoch, world=self.comm.world_size,
                             rank=self.comm.rank, init_s=round(time.time() - t0, 4))
            try:
                self._sync_state()
            except (CommAborted, RuntimeError) as e:
                if self.rdzv is None or not (self.comm.aborted or self.rdzv.aborted(self.comm.epoch)
                                             or _is_comm_error(e)):
                    raise
                self.events.emit("epoch_skipped", epoch=self.comm.epoch, during="state_sync")
                self.comm.abort()
                continue
            self.ddp.set_comm(self.comm)
            self.events.emit("state_synced", epoch=self.comm.epoch, step=self.step)
            return

    def _build_comm(self, a):
        """Arrival barrier, then construct + warm up the epoch's communicator.

        Process-group construction blocks inside C++ while holding the GIL, so
        we first wait — with non-blocking store polls that notice an abort —
        until every member has arrived; the construction itself then completes
        promptly.  It still runs in a helper thread as a second line of defence.
        """
        self.rdzv.kv.add(f"rdzv/arrive/{a.epoch}", 1)
        while self.rdzv.kv.counter(f"rdzv/arrive/{a.epoch}") < a.world:
            if self.rdzv.aborted(a.epoch):
                return None
            time.sleep(0.002)
        box = {}

        def build():
            try:
                c = Communicator(self._store, a.rank, a.world, a.epoch, device=self.device, job=self.ctx.job)
                c.warmup()
                box["comm"] = c
            except Exception as e:  # noqa: BLE001 - reported through box
                box["err"] = e

        th = threading.Thread(target=build, name=f"edl-comm-e{a.epoch}", daemon=True)
        th.start()
        while th.is_alive():
            th.join(0.02)
            if th.is_alive() and self.rdzv.aborted(a.epoch):
                return None  # abandon: the thread times out on its own
        if "err" in box:
            if self.rdzv.aborted(a.epoch) or _is_comm_error(box["err"]):
                return None
            raise box["err"]
        c = box["comm"]
        if self.rdzv.aborted(a.epoch):
            c.abort()
            return None
        return c

    def _state_tensors(self) -> list[torch.Tensor]:
        ts = [g.data for g in self.flat.groups]
        ts += list(self.opt.state_tensors().values())
        return ts

    def _sync_state(self):
        """Make every rank hold the newest committed state."""
        c = self.comm
        if c.world_size == 1:
            if self.needs_state and self.checkpoint is not None:
                self._maybe_restore()
            self.needs_state = False
            return
        have = -1 if self.needs_state else self.step
        max_step = int(c.ctrl_all_reduce([have], dist.ReduceOp.MAX)[0])
        if max_step < 0:
            # nobody holds trained state: fresh start (or checkpoint restore on rank 0)
            if c.rank == 0 and self.checkpoint is not None:
                self._maybe_restore()
            src_rank = 0
        else:
            cand = c.rank if (not self.needs_state and self.step == max_step) else 1 << 30
            src_rank = int(c.ctrl_all_reduce([cand], dist.ReduceOp.MIN)[0])
        differ = 1 if (self.needs_state or self.step != max_step) else 0
        need = int(c.ctrl_all_reduce([differ], dist.ReduceOp.MAX)[0])
        if need or max_step < 0:
            t0 = time.time()
            for t in self._state_tensors():
                c.broadcast(t, src_rank)
            scal = c.ctrl_broadcast([self.step, self.opt.step_count], src_rank)
            self.step = int(scal[0])
            self.opt.step_count = int(scal[1])
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)
            nbytes = sum(t.numel() * t.element_size() for t in self._state_tensors())
            self.events.emit("state_broadcast", src=src_rank, bytes=nbytes, s=round(time.time() - t0, 4))
        self.needs_state = False

    def _maybe_restore(self):
        if self.checkpoint is None:
            return
        st = self.checkpoint.restore_latest(self)
        if st is not None:
            self.events.emit("restored", step=self.step, source=st)

    # ------------------------------------------------------------------ steps
    def _micro_batches(self, data, plan: ElasticBatchPlan):
        rank = self.comm.rank
        world = self.comm.world_size
        return plan.indices(self.step, rank, world)

    def _run_step(self, loss_fn, data, plan):
        mbs = self._micro_batches(data, plan)
        self.flat.zero_grad()
        total = 0.0
        loss_acc = None
        for i, idx in enumerate(mbs):
            batch = data.batch(idx, self.device)
            w = len(idx) / plan.global_batch
            ctxm = self.ddp.no_sync() if i < len(mbs) - 1 else _null()
            with ctxm, trace.range(f"microbatch{i}"):
                with trace.range("fwd"):
                    loss = loss_fn(self.model, batch)
                with trace.range("bwd"):
                    (loss * w).backward() if w != 1.0 else loss.backward()
            ld = loss.detach() * w
            loss_acc = ld if loss_acc is None else loss_acc + ld
            total += w
        # a rank without samples (world > batch) still joins every all-reduce with zeros:
        # finish() zero-fills untouched gradients before flushing the buckets.
        with trace.range("grad_sync"):
            self.ddp.finish()
        self.fault.maybe_inject("after_backward", self.step, trainer=self)
        return None if loss_acc is None else loss_acc / total

    def _sync_point(self) -> bool:
        """Host-side completion of every gradient all-reduce; False if the epoch broke."""
        if self.device.type == "cuda":
            torch.cuda.current_stream(self.device).synchronize()
        return not self.comm.aborted

    def fit(self, loss_fn, data, num_steps: int, on_step=None) -> "ElasticTrainer":
        """Train until ``num_steps`` committed steps.  ``loss_fn(model, batch) -> scalar loss``."""
        gb = self.global_batch
        if gb is None:
            w = self.ctx.static_world or 1
            gb = w * self.micro_batch
            self.global_batch = gb
        plan = ElasticBatchPlan(len(data), gb, self.micro_batch, seed=17)
        self._connect()
        self._start_watchdog()
        try:
            self._enter_epoch()
            while self.step < num_steps:
                t0 = time.perf_counter()
                ok = True
                loss = None
                try:
                    self.fault.maybe_inject("step_start", self.step, trainer=self)
                    loss = self._run_step(loss_fn, data, plan)
                    ok = self._sync_point()
                except CommAborted as e:
                    log.warning("step %d aborted: %s", self.step, e)
                    ok = False
                except RuntimeError as e:
                    if self.comm is not None and (self.comm.aborted or _is_comm_error(e)):
                        log.warning("step %d failed in communication: %s", self.step, e)
                        ok = False
                    else:
                        raise
                if self.rdzv is not None:
                    apply, latest = self.rdzv.commit(self.comm.epoch, self.step, self.comm.world_size, ok,
                                                     gc=self.comm.rank == 0)
                else:
                    apply, latest = ok, 0
                if apply:
                    if self.checkpoint is not None:
                        self.checkpoint.fence()  # never update params under an in-flight snapshot
                    with trace.range("optimizer"):
                        self.opt.step(pre_scale=1.0)
                    self.step += 1
                    self.last_loss = loss
                    rec = {"step": self.step, "epoch": self.comm.epoch, "world": self.comm.world_size,
                           "dt": time.perf_counter() - t0}
                    self.history.append(rec)
                    self.events.emit("step_done", step=self.step, epoch=self.comm.epoch,
                                     world=self.comm.world_size)
                    self.metrics.record(self.step, rec["dt"], samples=self.global_batch,
                                        tokens=self.global_batch * self.tokens_per_sample, world=self.comm.world_size,
                                        loss=None)
                    if self.checkpoint is not None:
                        self.checkpoint.on_step(self)
                    if on_step is not None:
                        on_step(self, loss)
                    if self.log_every and self.step % self.log_every == 0 and self.comm.rank == 0:
                        log.info("step %d loss %.4f world %d", self.step, float(loss), self.comm.world_size)
                else:
                    self.events.emit("step_dropped", step=self.step, epoch=self.comm.epoch)
                if self.rdzv is not None and self.rdzv.plan_version != self.plan_version:
                    self._apply_runtime_plan(self.rdzv.plan_version)
                need_new = (not ok) or self.comm.aborted or (self.rdzv is not None and latest > self.comm.epoch)
                if need_new:
                    self._reconfigure()
        finally:
            self._stop.set()
        return self

    def _apply_runtime_plan(self, version: int) -> None:
        """Brain runtime knobs, switched by every rank at the same committed step."""
        self.plan_version = version
        mb = self.kv.get("plan/bucket_mb")
        if mb and float(mb) != self.ddp.bucket_mb:
            self.ddp.set_bucket_mb(float(mb))
            self.events.emit("plan_bucket_mb", mb=float(mb), step=self.step)
        ci = self.kv.get("plan/ckpt_interval")
        if ci and self.checkpoint is not None:
            self.checkpoint.interval = max(1, int(ci))

    def _reconfigure(self):
        old = self.comm
        self.events.emit("reconfigure", epoch=old.epoch, aborted=old.aborted)
        if old.aborted:
            pass
        else:
            old.shutdown()
        if self.rdzv is not None and self.rdzv.kv.exists(f"rdzv/leave/{self.ctx.node_id}"):
            raise SystemExit(0)
        self._enter_epoch()

    def close(self):
        self._stop.set()
        if self.rdzv is not None:
            try:
                self.rdzv.leave()  # finished: not a failure
            except Exception:
                pass
            self.rdzv.stop_heartbeat()
            if self.rdzv._hb is not None:
                self.rdzv._hb.join(timeout=5)
        if self._watchdog is not None:
            self._watchdog.join(timeout=5)
        if self._manager is not None:
            self._manager.stop()
        if self.comm is not None and not self.comm.aborted:
            self.comm.shutdown()


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def _is_comm_error(e: Exception) -> bool:
    s = str(e).lower()
    return any(k in s for k in ("nccl", "rccl", "gloo", "connection", "socket", "peer", "aborted", "timed out"))
