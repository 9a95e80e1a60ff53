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

import json
import logging
import os
import threading
import time
import weakref

import torch
import torch.distributed as dist

from easydl_amd.master.rendezvous import JobFinished, RendezvousClient, RendezvousConfig, RendezvousManager
from easydl_amd.master.store import KV, make_tcp_store
from easydl_amd.optim import FlatAdamW, FlatSGD, LRSchedule
from easydl_amd.parallel.comm import CommAborted, Communicator, LocalCommunicator, build_mesh
from easydl_amd.parallel.ddp import ElasticDDP
from easydl_amd.parallel.flat import FlatBuffers, FlatParams
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
                 grad_dtype=None, ctx: TrainerContext | None = None, seed: int = 1234,
                 schedule: LRSchedule | None = None,
                 rdzv_config: RendezvousConfig | None = None, checkpoint=None, log_every: int = 0,
                 store=None, tp: int | None = None, moment_dtype: str = "fp32"):
        self.ctx = ctx or TrainerContext.from_env()
        hang = float(os.environ.get("EDL_HANG_DUMP_S", 0) or 0)
        if hang > 0:   # diagnostics: every thread's Python stack to stderr every `hang` seconds
            import faulthandler
            faulthandler.dump_traceback_later(hang, repeat=True)
        if device is None:
            if torch.cuda.is_available():
                device = torch.device("cuda", self.ctx.gpu or 0)
            else:
                device = torch.device("cpu")
        self.device = torch.device(device)
        t_init = time.perf_counter()
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
            torch.empty(1, device=self.device)  # HIP context now, so its cost shows up in the timeline
        self.resources = apply_plan(self.ctx, self.device)  # Brain CU mask / HBM cap
        if self.device.type == "cuda":
            from easydl_amd.ops import gemm_tuning
            self.gemm_tuning = gemm_tuning.apply()  # shipped TunableOp selections (or tune / off)
        if self.device.type == "cuda" and torch.cuda.current_stream(self.device).cuda_stream == 0:
            # never compute on the legacy NULL stream: it implicitly serialises with every
            # blocking stream, e.g. the CU-masked snapshot copy stream (ckpt/manager.py)
            self.compute_stream = torch.cuda.Stream(self.device)
            torch.cuda.set_stream(self.compute_stream)
        self.events = EventLog(os.path.join(self.ctx.run_dir, f"events-{self.ctx.role}{self.ctx.index}.jsonl"),
                               proc=f"{self.ctx.role}{self.ctx.index}")
        try:
            ncpu = len(os.sched_getaffinity(0))
        except (AttributeError, OSError):
            ncpu = os.cpu_count()
        self.events.emit("device_ready", s=round(time.perf_counter() - t_init, 4), cpus=ncpu,
                         threads=torch.get_num_threads())
        from easydl_amd.utils.kmix import KernelMixMeter
        self.kmix = KernelMixMeter(self.device)    # live compute / bandwidth split for the Brain
        if optimizer not in ("adamw", "sgd"):
            raise ValueError(f"unknown optimizer {optimizer}")
        self._model_fn, self._seed = model_fn, seed
        if moment_dtype not in ("fp32", "bf16", "auto"):
            raise ValueError(f"moment_dtype must be fp32, bf16 or auto, got {moment_dtype}")
        self._opt_args = dict(optimizer=optimizer, lr=lr, weight_decay=weight_decay, betas=betas, momentum=momentum,
                              max_grad_norm=max_grad_norm, schedule=schedule, grad_dtype=grad_dtype,
                              bucket_mb=bucket_mb, moment_dtype=moment_dtype)
        self.checkpoint = checkpoint
        # tensor parallelism (Megatron layout inside each DP replica): model_fn(device, tp_group);
        # the model is built at the first epoch, once this process's TP rank is known
        self.tp = int(tp if tp is not None else os.environ.get("EDL_TP", 1))
        self.tp_group = None
        self.held_tp = None          # TP rank whose parameter shard this process holds
        self.ckpt_tag = ""
        self.dp_comm = None
        self.comm = None
        self.model = self.flat = self.bufs = self.opt = self.ddp = None
        if self.tp == 1:
            self._build_model(0)
        else:
            from easydl_amd.parallel.tp import TPGroup
            self.tp_group = TPGroup(size=self.tp, sequence_parallel=os.environ.get("EDL_SP", "0") == "1")
        self.global_batch = global_batch
        self.micro_batch = micro_batch
        self.step = 0                # committed optimizer steps
        self._warm_windows: set = set()   # (standby, request id) warm-up windows granted
        self._warm_published = False
        self._act_published = False
        self._rehomed = False        # state adopted from a dead worker moved into own memory (_maybe_rehome)
        self.needs_state = True     # fresh process: must receive state unless everyone is fresh
        self.comm = None
        self.assignment = None
        self.checkpoint = checkpoint
        self.log_every = log_every
        self._phases = os.environ.get("EDL_STEP_PHASES", "0") == "1"
        self._step_sync = self._phases or os.environ.get("EDL_STEP_SYNC", "0") == "1"
        self._marks = None          # step-mark page (utils/stepmarks.py), opened in fit()
        self._sync_next = True
        self.rdzv_config = rdzv_config
        self._store = store
        self._manager = None
        self._watchdog = None
        self._prejoin = None   # fit(): warm-up run by a process joining a running job
        self._stop = threading.Event()
        self.fault = fault.FaultInjector.from_env(self.ctx, self.events)
        self.history: list[dict] = []
        self.last_loss = None
        self.tokens_per_sample = 0
        self.metrics = MetricsReporter(
            path=os.path.join(self.ctx.run_dir, f"metrics-{self.ctx.role}{self.ctx.index}.jsonl"))
        self.plan_version = 0
        self._stop_requested = False
        self._master_lost: str | None = None    # set by the watchdog (see _start_watchdog)
        self._mb_split = 1           # >1: micro-batches split while a takeover waits for HBM (_memory_plan)
        self._mb_recompute = None    # not None: the model's recompute flag to restore (_memory_plan)
        self._shadow_stream = None   # gradient shadow copies (_shadow_grads)
        self._shadow_pending = False
        self._shadow_resume = None   # {"step", "mb", "host"}: resume that step at that micro-batch
        self._hshadow = None         # host gradient shadow (utils/gshadow.py), when HBM has no room
        self._opt_stream = None      # optimizer update overlapping the next forward (_opt_overlap)
        self._opt_overlap_off = False
        self._act_need = 0

    def request_stop(self) -> None:
        """End ``fit`` after the current step (from ``on_step``).  Every rank must ask at the
        same committed step, e.g. from a step-based condition, like any other collective
        decision."""
        self._stop_requested = True

    # ------------------------------------------------------------------ setup
    def _build_model(self, tp_rank: int) -> None:
        a = self._opt_args
        t0 = time.perf_counter()
        torch.manual_seed(self._seed + 1009 * tp_rank)  # DP replicas of a shard initialise identically
        if self.tp > 1:
            self.tp_group.rank = tp_rank
            self.model = self._model_fn(self.device, self.tp_group)
        else:
            self.model = self._model_fn(self.device)
        t1 = time.perf_counter()
        self.flat = FlatParams(self.model, weight_decay=a["weight_decay"], grad_dtype=a["grad_dtype"])
        self.bufs = FlatBuffers(self.model)
        if a["optimizer"] == "adamw":
            self.opt = FlatAdamW(self.flat, lr=a["lr"], betas=a["betas"], weight_decay=a["weight_decay"],
                                 max_grad_norm=a["max_grad_norm"], schedule=a["schedule"],
                                 moment_dtype=self._choose_moment_dtype(a["moment_dtype"]))
        else:
            self.opt = FlatSGD(self.flat, lr=a["lr"], momentum=a["momentum"], weight_decay=a["weight_decay"],
                               max_grad_norm=a["max_grad_norm"], schedule=a["schedule"])
        self._agree_moment_dtype()    # store known (TP: built at the first epoch): publish / adopt now
        if self.tp > 1:
            # grad norm over the whole model: replicated groups (norms) count once
            w = []
            for g in self.flat.groups:
                rep = {bool(getattr(sl.param, "_tp_replicated", False)) for sl in g.slots}
                if len(rep) != 1:
                    raise ValueError(f"flat group {g.name} mixes TP-replicated and sharded parameters")
                w.append(1.0 / self.tp if rep.pop() else 1.0)
            self.opt.norm_weights = w
            self.opt.norm_reduce = lambda t: self.comm.tp.all_reduce(t)
        self.ddp = ElasticDDP(self.flat, None, bucket_mb=a["bucket_mb"])
        from easydl_amd.utils import vram
        dropped = vram.release_unused()   # adopted buffers nothing here took: back to the driver
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        if getattr(self, "events", None) is not None:
            self.events.emit("model_built", model_s=round(t1 - t0, 4), flat_opt_s=round(time.perf_counter() - t1, 4),
                             adopted=len(vram.TAKEN), adopted_unused=len(dropped))
            if dropped:
                log.warning("vram: %d adopted buffers matched nothing and were released: %s", len(dropped),
                            dropped[:8])

    def _choose_moment_dtype(self, want: str) -> torch.dtype:
        """``auto``: bf16 moments exactly when the host DRAM budget of this rank (ckpt/manager.py
        host_budget_bytes) holds two FULL snapshot slots with bf16 moments but not with fp32 ones
        -- e.g. a Llama-3-70B TP=8 shard on an 8-GPU node: 2 x 106 GB > 151 GB >= 2 x 71 GB --
        so the in-memory snapshots keep the Adam moments instead of going lean (a lean restore
        restarts them).  The state of a DP replica is sharded over the DP group."""
        if want != "auto":
            return torch.bfloat16 if want == "bf16" else torch.float32
        from easydl_amd.utils import vram
        inherited = vram.adopted_dtype("opt/", "/m")
        if inherited is not None:
            # a takeover keeps the dead worker's (job-agreed) choice: its moments are adopted as they are
            return inherited
        agreed = self._job_moment_dtype()
        if agreed is not None:
            return agreed
        ck = self.checkpoint
        if ck is None or not hasattr(ck, "host_budget_bytes"):
            return torch.float32
        dp = 1
        if self.comm is not None:
            dp = getattr(getattr(self.comm, "dp", None), "world_size", None) or (self.comm.world_size // self.tp)
        elif self.ctx.static_world:
            dp = max(1, self.ctx.static_world // self.tp)
        n = sum(g.numel for g in self.flat.groups)
        bufs = sum(t.numel() * t.element_size() for t in self.bufs.tensors.values())
        full32, full16 = (n * 12 + bufs) / dp, (n * 8 + bufs) / dp
        budget = ck.host_budget_bytes(self)
        pick = torch.bfloat16 if 2 * full32 > budget >= 2 * full16 else torch.float32
        if getattr(self, "events", None) is not None:
            self.events.emit("moment_dtype", dtype=str(pick).replace("torch.", ""), budget_bytes=int(budget),
                             full_fp32_bytes=int(full32), full_bf16_bytes=int(full16),
                             budget_gb=round(budget / 2**30, 2), full_fp32_gb=round(full32 / 2**30, 3))
        return pick

    _MOMENT_KEY = "job/moment_dtype"

    def _job_moment_dtype(self) -> torch.dtype | None:
        """The moment dtype this job already decided (job store), None before the first decision."""
        kv = getattr(self, "kv", None)
        if kv is None:
            return None
        v = kv.get_str(self._MOMENT_KEY)
        return None if v is None else (torch.bfloat16 if v == "bf16" else torch.float32)

    def _agree_moment_dtype(self) -> None:
        """``moment_dtype="auto"`` is decided once per JOB, not per process: the first process to
        reach the store publishes its pick (compare-and-set) and every later one -- a replacement
        started while the dead worker's segments still fill /dev/shm, a rank on a busier node --
        adopts it.  Otherwise a state transfer or snapshot restore would copy raw moment bytes
        into buffers of another dtype (ckpt/manager.py _load_shard now refuses that loudly)."""
        if (self._opt_args["moment_dtype"] != "auto" or getattr(self, "kv", None) is None
                or not hasattr(self.opt, "set_moment_dtype")):
            return
        mine = "bf16" if self.opt.moment_dtype == torch.bfloat16 else "fp32"
        got = self.kv.compare_set(self._MOMENT_KEY, "", mine) or mine
        if got != mine:
            self.opt.set_moment_dtype(torch.bfloat16 if got == "bf16" else torch.float32)
            self.events.emit("moment_dtype", dtype=got, adopted_from_job=True, local_pick=mine)

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
        if self.opt is not None:
            self._agree_moment_dtype()     # (TP models are built later, with the store already known)
        if self.ctx.embedded_master and self.ctx.index == 0:
            cfg = self.rdzv_config or RendezvousConfig(min_nodes=self.ctx.static_world,
                                                       max_nodes=self.ctx.static_world, granule=self.tp)
            self._manager = RendezvousManager(self.kv, cfg, events=self.events)
            self._manager.start()
        info = {"index": self.ctx.index, "role": self.ctx.role, "gpu": self.ctx.gpu}
        self.rdzv = RendezvousClient(self.kv, self.ctx.node_id, info)
        self.metrics.kv, self.metrics.node = self.kv, self.ctx.node_id
        if self._prejoin is not None and self._job_is_running():
            self.rdzv.arriving()
            self._prejoin()
        self.rdzv.join()
        self.events.emit("joined", node=self.ctx.node_id)

    def _job_is_running(self) -> bool:
        """A live epoch exists: this process is a scale-up joiner or a replacement beside
        survivors (not part of the initial cohort, not a restore with nobody left)."""
        e = self.rdzv.latest_epoch()
        return e > 0 and not self.rdzv.aborted(e) and not self.kv.exists("train/done")

    def _prejoin_warmup(self, loss_fn, data, plan) -> None:
        """One local forward + backward on this process's own (not yet synced) weights
        BEFORE it announces itself.  A fresh process's first iteration loads every
        kernel (MIOpen convolutions, hipBLASLt, our extensions) and grows the caching
        allocator: measured 1.5 s for ResNet-50 joiners, during which the running world
        stalled in its first collective with them (profiles/r02_scale_up_resnet50_*).
        Here the running world keeps training meanwhile.  No communicator exists yet,
        so no collective is issued; the gradients are discarded."""
        if self.model is None or self.tp > 1:
            return
        t0 = time.perf_counter()
        idx = plan.indices(0, 0, 1)[0]
        self.flat.zero_grad()
        loss = loss_fn(self.model, data.batch(idx, self.device))
        loss.backward()
        # every real step starts with zero_grad(): fresh gradient window and a new weight
        # generation, so transposed-weight caches built from these random weights are dropped
        self.flat.zero_grad()
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        self.events.emit("prejoin_warmup", s=round(time.perf_counter() - t0, 4))

    def _start_watchdog(self):
        """Abort the epoch's communicators as soon as the master flags the epoch broken.  A
        store that stays unreachable for ``EDL_MASTER_TIMEOUT_S`` (default 60 s) means the job
        master is gone: the epoch is aborted too (no collective waits forever) and the step
        loop raises :class:`MasterUnreachable` instead of re-forming (there is nobody to
        re-form with); the operator then replaces the whole job's processes."""
        limit = float(os.environ.get("EDL_MASTER_TIMEOUT_S", 60))

        def loop():
            first_fail = None
            while not self._stop.wait(0.01):
                c = self.comm
                if c is None or self.rdzv is None:
                    continue
                if c.aborted and first_fail is None:
                    continue
                try:
                    if self.rdzv.aborted(c.epoch):
                        self.events.emit("abort_seen", epoch=c.epoch)
                        c.abort()
                    if first_fail is not None:
                        self.events.emit("store_reachable", after_s=round(time.monotonic() - first_fail, 3))
                    first_fail = None
                except Exception as e:  # noqa: BLE001 - classified below, never swallowed for good
                    now = time.monotonic()
                    if first_fail is None:
                        first_fail = now
                        self.events.emit("store_unreachable", error=f"{type(e).__name__}: {e}"[:200])
                    elif now - first_fail > limit and self._master_lost is None:
                        self._master_lost = f"{type(e).__name__}: {e}"[:300]
                        self.events.emit("master_lost", after_s=round(now - first_fail, 3), error=self._master_lost)
                        log.error("job master store unreachable for %.0f s: %s", now - first_fail, e)
                        try:
                            c.abort()
                        except Exception:  # noqa: BLE001
                            pass
                        return

        self._watchdog = threading.Thread(target=loop, name="edl-watchdog", daemon=True)
        self._watchdog.start()

    def _enter_epoch(self):
        """Join the next live epoch; retries when the epoch breaks while it is being built."""
        self.wait_update()      # the state may be sent to a joiner, snapshotted or restored next
        self._sync_next = True
        while True:
            t0 = time.time()
            if self.rdzv is None:
                self.comm = LocalCommunicator(self.device)
                self.assignment = None
            else:
                a = self.rdzv.wait_assignment(after_epoch=self.assignment.epoch if self.assignment else 0)
                self.assignment = a
                self.events.emit("epoch_joined", epoch=a.epoch, rank=a.rank, world=a.world, reason=a.reason)
                if a.world == 1 and self.tp == 1:
                    self.comm = LocalCommunicator(self.device, epoch=a.epoch)
                else:
                    comm = self._build_comm(a)
                    if comm is None:
                        self.events.emit("epoch_skipped", epoch=a.epoch)
                        continue
                    self.comm = comm
            self.events.emit("comm_ready", epoch=self.comm.epoch, world=self.comm.world_size,
                             rank=self.comm.rank, init_s=round(time.time() - t0, 4))
            if self.tp > 1:
                if self.rdzv is None:
                    raise RuntimeError("tensor parallelism needs a rendezvous (tp > 1 ranks)")
                if self.model is None:
                    self._build_model(self.comm.tp_rank)
                self.tp_group.rebind(self.comm.tp)
                self.dp_comm = self.comm.dp
            else:
                self.dp_comm = self.comm
            try:
                self._sync_state() if self.tp == 1 else self._sync_state_tp()
                if self.checkpoint is not None and hasattr(self.checkpoint, "prepare_layout"):
                    # snapshot mode (full / lean / off) of the new layout: agreed here, where a
                    # dead peer means "skip this epoch", never inside a step's snapshot
                    self.checkpoint.prepare_layout(self)
            except (CommAborted, RuntimeError) as e:
                if self.rdzv is None or not (self.comm.aborted or self.rdzv.aborted(self.comm.epoch)
                                             or _is_comm_error(e)):
                    raise
                self.events.emit("epoch_skipped", epoch=self.comm.epoch, during="state_sync")
                self.comm.abort()
                continue
            self.events.emit("state_transferred", epoch=self.comm.epoch, step=self.step)
            if self.rdzv is not None:
                try:
                    self._publish_probe()
                    self._agree_runtime_plan()   # may adopt the Brain's policy for a deferred probe
                except (CommAborted, RuntimeError) as e:
                    if not (self.comm.aborted or self.rdzv.aborted(self.comm.epoch) or _is_comm_error(e)):
                        raise
                    self.events.emit("epoch_skipped", epoch=self.comm.epoch, during="runtime_plan")
                    self.comm.abort()
                    continue
            # binds the epoch's comm (registers the gradient buffers if the agreed policy routes
            # them to the xGMI engine)
            self.ddp.set_comm(self.dp_comm)
            xg = getattr(self.dp_comm, "xgmi", None)
            mem = {}
            if self.device.type == "cuda":
                free, total = torch.cuda.mem_get_info(self.device)
                mem = {"gpu_free_gb": round(free / 2**30, 1), "reserved_gb":
                       round(torch.cuda.memory_reserved(self.device) / 2**30, 1)}
            self._memory_plan()
            self.events.emit("state_synced", epoch=self.comm.epoch, step=self.step, **mem,
                             grad_buffers_mapped=len(getattr(xg, "_registered", ())) if xg is not None else 0,
                             probe_pending=[g for g, c in self._comm_groups() if getattr(c, "probe_pending", False)])
            return

    def _comm_groups(self):
        """(name, communicator) of this rank's data-plane groups: DP, and TP when sharded."""
        out = [("dp", self.dp_comm)]
        if self.tp > 1 and getattr(self.comm, "tp", None) is not None:
            out.append(("tp", self.comm.tp))
        return out

    def _publish_probe(self) -> None:
        """The epoch's RCCL-vs-engine tables go to the Brain (``comm/probe/<group>``), one
        per group, written by the group's rank 0."""
        for group, c in self._comm_groups():
            probe = getattr(c, "xgmi_probe", None)
            if probe and c.rank == 0:
                if not probe.get("cached") and probe.get("source") != "brain":   # new measurements only
                    doc = {"epoch": self.comm.epoch, "world": c.world_size, "group": group, "probe": probe}
                    self.kv.set(f"comm/probe/{group}", json.dumps(doc))
                self.events.emit("allreduce_probe", epoch=self.comm.epoch, group=group, world=c.world_size,
                                 selected=probe.get("selected"), policy=probe.get("policy"),
                                 cached=bool(probe.get("cached")), source=probe.get("source", "probe"),
                                 probe_s=probe.get("probe_s"), engine_blocks=probe.get("engine_blocks"))

    def _agree_runtime_plan(self) -> None:
        """Every rank of the new epoch switches to the same runtime plan: the highest plan
        version any of them sees.  Joiners and survivors re-apply it alike, so the
        Brain's all-reduce policy (which the epoch's own probe just replaced) holds
        on every rank, not only on the survivors."""
        seen = float(self.kv.counter("plan/version"))
        v = int(self.comm.ctrl_all_reduce([seen], dist.ReduceOp.MAX)[0])
        if v > 0:
            self._apply_runtime_plan(v)

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
                _join_releases()
                # a job's first epoch may measure the all-reduce policy; every later epoch
                # (shrink, rejoin, scale-up) is on the recovery critical path: cached policy or
                # RCCL until the deferred probe after its first committed step
                probe = "now" if a.reason == "initial" else "defer"
                if self.tp > 1:
                    c = build_mesh(self._store, a.rank, a.world, a.epoch, self.tp, device=self.device,
                                   job=self.ctx.job, probe=probe)
                else:
                    c = Communicator(self._store, a.rank, a.world, a.epoch, device=self.device, job=self.ctx.job,
                                     probe=probe)
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
        ts += list(self.bufs.tensors.values())
        return ts

    def _sync_state(self):
        """Make every rank hold the newest committed state."""
        c = self.comm
        if c.world_size == 1:
            if self.needs_state:
                # nobody to send the state to: the moments may arrive under the first step
                self._maybe_restore(defer_moments=True)
            self.needs_state = False
            self._state_settled()
            return
        if self.checkpoint is not None:
            # a world-1 restore may still be copying its moments (deferred under the first step);
            # this rank may now send its state to others: it must hold all of it
            self.checkpoint.complete_restore()
        have = -1 if self.needs_state else self.step
        max_step = int(c.ctrl_all_reduce([have], dist.ReduceOp.MAX)[0])
        holder = max_step >= 0 and not self.needs_state and self.step == max_step
        if max_step < 0:
            # nobody holds trained state: fresh start (or checkpoint restore on rank 0)
            if c.rank == 0:
                self._maybe_restore()
            holders = [0]
        else:
            onehot = [0.0] * c.world_size
            onehot[c.rank] = 1.0 if holder else 0.0
            holders = [r for r, v in enumerate(c.ctrl_all_reduce(onehot, dist.ReduceOp.MAX).tolist()) if v > 0]
        src_rank = holders[0]
        if len(holders) < c.world_size or max_step < 0:
            t0 = time.time()
            self._fence_snapshot_before_overwrite(c, src_rank, holder)
            # every up-to-date rank sends a slice (SURVEY.md §2.8 multi-source scatter):
            # a joiner's inbound traffic is spread over one link per survivor
            c.transfer_state(self._state_tensors(), holders if max_step >= 0 else [src_rank])
            scal = c.ctrl_broadcast([self.step, self.opt.step_count, getattr(self.opt, "moment_origin", 0)],
                                    src_rank)
            self.step = int(scal[0])
            self.opt.step_count = int(scal[1])
            if hasattr(self.opt, "moment_origin"):
                self.opt.moment_origin = int(scal[2])
            if self.device.type == "cuda":
                torch.cuda.current_stream(self.device).synchronize()
            nbytes = sum(t.numel() * t.element_size() for t in self._state_tensors())
            self.events.emit("state_broadcast", src=src_rank, sources=len(holders), bytes=nbytes,
                             s=round(time.time() - t0, 4))
        self.needs_state = False
        self._state_settled()

    def _fence_snapshot_before_overwrite(self, c, src: int, holder: bool) -> None:
        """A state transfer rewrites this rank's buffers unless it is the source, or a
        holder of the same step (multi-source transfer never writes holders; an RCCL
        broadcast writes identical bytes).  The xGMI-only broadcast (TP groups)
        zero-fills non-source ranks first.  If the buffers will change, the
        in-flight snapshot D2H (which reads them on the checkpoint engine's stream) must
        finish first, or its slot would mix old and new bytes under the old checksum.
        The fence is a stream wait, not a host block."""
        if self.checkpoint is None or self.device.type != "cuda" or c.rank == src:
            return
        if not holder or getattr(c, "backend", "") == "xgmi":
            self.checkpoint.fence()

    def _sync_state_tp(self):
        """DP x TP state agreement.  Each TP rank's shard is replicated over its
        DP group: if every group still has a member holding its shard at the
        newest committed step, that member broadcasts inside the group (only
        new or re-ranked processes receive).  If some shard has no live holder
        (e.g. TP = world and a worker died), every rank rolls back to the
        newest snapshot step that all shards have in memory."""
        c = self.comm
        t = c.tp_rank
        valid = (not self.needs_state) and self.held_tp == t
        max_step = int(c.ctrl_all_reduce([-1 if self.needs_state else self.step], dist.ReduceOp.MAX)[0])
        mine_ok = 1 if (valid and self.step == max_step) else 0
        grp_ok = int(c.dp.ctrl_all_reduce([mine_ok], dist.ReduceOp.MAX)[0]) if c.dp.world_size > 1 else mine_ok
        all_ok = int(c.ctrl_all_reduce([grp_ok], dist.ReduceOp.MIN)[0])
        self.ckpt_tag = f"-t{t}of{self.tp}"
        if max_step >= 0 and all_ok:
            if c.dp.world_size > 1 and int(c.dp.ctrl_all_reduce([1 - mine_ok], dist.ReduceOp.MAX)[0]):
                # every DP-group member holding this shard at the newest step sends a slice
                # (multi-source): the replacement's inbound traffic is spread over
                # one link per holder instead of one source's single link
                onehot = [0.0] * c.dp.world_size
                onehot[c.dp.rank] = float(mine_ok)
                holders = [r for r, v in enumerate(c.dp.ctrl_all_reduce(onehot, dist.ReduceOp.MAX).tolist())
                           if v > 0]
                src = holders[0]
                t0 = time.time()
                self._fence_snapshot_before_overwrite(c.dp, src, bool(mine_ok))
                c.dp.transfer_state(self._state_tensors(), holders)
                scal = c.dp.ctrl_broadcast([self.step, self.opt.step_count,
                                            getattr(self.opt, "moment_origin", 0)], src)
                self.step, self.opt.step_count = int(scal[0]), int(scal[1])
                if hasattr(self.opt, "moment_origin"):
                    self.opt.moment_origin = int(scal[2])
                if self.device.type == "cuda":
                    torch.cuda.current_stream(self.device).synchronize()
                nbytes = sum(x.numel() * x.element_size() for x in self._state_tensors())
                self.events.emit("state_broadcast", src=src, sources=len(holders), group="dp", tp_rank=t,
                                 bytes=nbytes, s=round(time.time() - t0, 4))
        else:
            mine = self.checkpoint.latest_step(self) if self.checkpoint is not None else -1
            target = int(c.ctrl_all_reduce([mine], dist.ReduceOp.MIN)[0])
            if target >= 0:
                src = self.checkpoint.restore_latest(self, max_step=target)
                if src is None or self.step != target:
                    raise RuntimeError(f"TP shard {t}: snapshot of step {target} not restorable")
                self.events.emit("restored", step=self.step, source=src, tp_rank=t)
            elif max_step >= 0:
                raise RuntimeError(f"TP shard {t} lost at step {max_step} and no in-memory snapshot covers it")
            else:
                # fresh start; replicas of a shard are identical by seeding (no broadcast)
                self._reinit_adopted()
        self.held_tp = t
        self.needs_state = False
        self._state_settled()

    def _open_marks(self) -> None:
        """Step-mark page of this worker slot (utils/stepmarks.py), with VRAM hand-over on.
        After an HBM resume the page still holds the dead worker's marks, which the post-reap
        check re-reads (ckpt/manager.py _check_marks_after_reap): this process writes its own
        only once that check has passed (the step loop calls this again after each fence).  If
        it dies before, its replacement finds marks of a writer it did not adopt from and
        restores from the snapshot."""
        from easydl_amd.utils import vram
        if self._marks is not None or not vram.enabled() or getattr(self, "kv", None) is None:
            return
        if self.checkpoint is not None and self.checkpoint.hbm_unverified():
            return
        from easydl_amd.utils.stepmarks import StepMarks
        try:
            self._marks = StepMarks(self.ctx.job, f"{self.ctx.role}{self.ctx.index}", device=self.device)
        except OSError as e:
            log.warning("step marks unavailable: %s", e)
            return
        self._settle_marks()

    def _settle_marks(self) -> None:
        """The state is settled at self.step (epoch entry: restore / transfer done)."""
        if self._marks is None:
            return
        if self.device.type == "cuda":
            torch.cuda.current_stream(self.device).synchronize()
        self._marks.set_now(self.step)

    def _publish_vram(self) -> None:
        """Export the persistent state buffers for the hot standby on this GPU (utils/vram.py):
        if this process dies, the standby builds on them instead of waiting for the driver to
        reclaim and re-allocate 128 GB (Llama-3-8B)."""
        from easydl_amd.utils import vram
        if not (vram.enabled() and self.device.type == "cuda" and getattr(self, "kv", None) is not None):
            return
        ts = self.vram_state_tensors()
        try:
            n = vram.publish(self.kv, f"{self.ctx.role}{self.ctx.index}", self.ctx.node_id, ts)
        except Exception as e:  # noqa: BLE001 - hand-over is an optimisation; training goes on
            log.warning("vram hand-over export failed: %s", e)
            return
        self.events.emit("vram_published", tensors=n, of=len(ts),
                         adopted=dict(vram.STATS, adopted_gb=round(vram.STATS["adopted_bytes"] / 2**30, 1)))

    def vram_state_tensors(self) -> dict[str, torch.Tensor]:
        """The persistent buffers a hot standby adopts (utils/vram.py names): flat weights and
        gradients, optimizer state, module buffers (BatchNorm running statistics)."""
        ts = {}
        for g in self.flat.groups:
            ts[f"flat/{g.name}/data"], ts[f"flat/{g.name}/grad"] = g.data, g.grad
        for g, st in zip(self.flat.groups, getattr(self.opt, "state", [])):
            for k, t in st.items():
                if isinstance(t, torch.Tensor) and t is not g.data:
                    ts[f"opt/{g.name}/{k}"] = t
        for k, t in getattr(self.bufs, "tensors", {}).items():
            ts[f"bufs/{k}"] = t
        ts.update(self.flat.shadow_tensors())
        return ts

    def _publish_warm_spec(self, data) -> None:
        """Tell the parked standby on this GPU what to warm up with (operator/standby.py
        warm_device): one layer of this model's width at this job's micro-batch shape, so the
        GEMM solutions, kernels and library handles of the replacement's first step are loaded
        before it is needed.  Published before this worker's first step, and the worker waits
        for that warm-up (bounded, ``EDL_WARM_WAIT_S``, default 60 s): a warm-up never runs
        beside a training step of this GPU, and it has the memory the step's activations will
        take later.  A standby that arrives later, with training running, warms up in a window
        the job master plans and every rank applies at one step (_warm_window)."""
        from easydl_amd.utils import vram
        if (self._warm_published or not vram.enabled() or self.device.type != "cuda"
                or getattr(self, "kv", None) is None):
            return
        self._warm_published = True
        from dataclasses import asdict

        from easydl_amd.models.llama import Llama
        seq = getattr(data, "seq", None)
        spec = None
        if isinstance(self.model, Llama) and self.tp == 1 and seq:
            cfg = {k: v for k, v in asdict(self.model.cfg).items() if isinstance(v, (bool, int, float))}
            cfg["n_layers"] = 1
            spec = {"model": "llama", "cfg": cfg, "batch": [self.micro_batch, int(seq)]}
        vram.publish_warm(self.kv, f"{self.ctx.role}{self.ctx.index}", spec)
        t0 = time.perf_counter()
        limit = float(os.environ.get("EDL_WARM_WAIT_S", 60))
        state = vram.standby_warm_on(self.kv, self.device.index)
        while state is False and time.perf_counter() - t0 < limit:
            time.sleep(0.05)
            state = vram.standby_warm_on(self.kv, self.device.index)
        if state is not None:
            self.events.emit("standby_warm_wait", s=round(time.perf_counter() - t0, 3), warm=bool(state))

    def _warm_window(self, ww: dict) -> None:
        """Runtime plan ``warm_window`` (master/main.py _grant_warm_windows): a standby that
        arrived while this job trains warms up on this rank's GPU now, between two steps --
        grant it and wait (bounded, EDL_WARM_WINDOW_S) for its warm key.  Every rank applies the
        plan at the same committed step; ranks on other GPUs go on and meet this one at the next
        collective.  A request that is gone (handled, or its standby took over) is skipped."""
        from easydl_amd.utils import vram
        name, gpu = ww.get("standby"), self.device.index
        if (self.device.type != "cuda" or gpu not in (ww.get("gpus") or []) or not name
                or (name, ww.get("id")) in self._warm_windows):
            return
        self._warm_windows.add((name, ww.get("id")))
        req = vram.read_warm_request(self.kv, name)
        if not req or req.get("id") != ww.get("id") or name not in vram.roster(self.kv):
            return
        t0 = time.perf_counter()
        self.kv.set(f"standby/warm_grant/{name}/gpu{gpu}", str(ww.get("id")))
        limit = float(os.environ.get("EDL_WARM_WINDOW_S", 60))
        next_roster = t0 + 0.5
        while not self.kv.exists(f"standby/warm/{name}/gpu{gpu}") and time.perf_counter() - t0 < limit:
            time.sleep(0.02)
            if time.perf_counter() > next_roster:     # a standby that took over or died ends the window
                next_roster = time.perf_counter() + 0.5
                if name not in vram.roster(self.kv):
                    break
        self.events.emit("standby_warm_window", standby=name, step=self.step, s=round(time.perf_counter() - t0, 3),
                         warm=self.kv.exists(f"standby/warm/{name}/gpu{gpu}"))

    def _publish_act(self) -> None:
        """HBM a step needs beyond the persistent state (activations, workspaces), after the
        first step: a replacement that adopts the state checks it against what the GPU has free
        (_memory_plan)."""
        from easydl_amd.utils import vram
        if (self._act_published or not vram.enabled() or self.device.type != "cuda"
                or getattr(self, "kv", None) is None):
            return
        if self._mb_split > 1 or self._mb_recompute is not None:
            return      # a memory-limited step's peak is not a full step's (_memory_plan)
        self._act_published = True
        # only this process's own allocations count against its allocator's peak: state adopted
        # from a dead worker is imported memory the caching allocator never reserved (counting it
        # published 0 for a replacement, and the next replacement would not have split its step)
        adopted = set(vram.TAKEN.values())
        persistent = sum(t.untyped_storage().nbytes() for t in self.vram_state_tensors().values()
                         if t.data_ptr() not in adopted)
        act = max(0, torch.cuda.max_memory_reserved(self.device) - persistent)
        vram.publish_act(self.kv, f"{self.ctx.role}{self.ctx.index}", act, self.micro_batch)
        self._maybe_shadow(act)

    def _maybe_shadow(self, act: int) -> None:
        """Turn the gradient shadow on after the first step if the GPU can afford it: a
        replacement starts with only the HBM this worker leaves free (the rest of its memory
        is reclaimed seconds after it dies), and its first step must still fit one sample per
        micro-batch there (_memory_plan).  At Llama-3-8B (2 x 8k tokens per micro-batch) the
        16 GB shadow does not fit that budget: the first step then blocked in hipMalloc and
        the time-to-recover doubled (profiles/r05_ttr_headline.md), so it stays off there."""
        if self.flat.gshadow is not None or not self._shadow_wanted():
            return
        from easydl_amd.utils import vram
        free = torch.cuda.mem_get_info(self.device)[0]
        if not vram.standby_warm_on(self.kv, self.device.index):
            # no warm standby on this GPU yet (a replacement before its refill arrives): keep the
            # room one will take (a context, the GEMM libraries' workspaces, its warm-up's cache)
            free -= int(float(os.environ.get("EDL_STANDBY_RESERVE_GB", "16")) * 2**30)
        shadow = sum(g.grad.untyped_storage().nbytes() for g in self.flat.groups)
        need = act / max(1, self.micro_batch) * 1.15
        mode = os.environ.get("EDL_GRAD_SHADOW", "1")
        # default: HBM where it fits, else none.  The host shadow is opt-in ("host"): at the 8B
        # headline its device -> host copies share the host link with the snapshots' (every 2
        # steps), so a kill right after a snapshot step found no finished copy, and the dead
        # worker's 30 GB of page-locked memory delayed its teardown and the replacement's first
        # step by ~0.3 s (profiles/r05_grad_shadow_ab.md)
        where = ("hbm" if mode == "force" or (mode != "host" and free - shadow >= need)
                 else "host" if mode == "host" else None)
        self.events.emit("grad_shadow", on=where is not None, where=where, gb=round(shadow / 2**30, 1),
                         free_gb=round(free / 2**30, 1), replacement_need_gb=round(need / 2**30, 1))
        if where is None:
            return
        if where == "hbm":
            self.flat.ensure_shadow(self._state_pool())
            self._publish_vram()
            return
        # host memory: the page-locked segment is created and registered off the step path; the
        # shadow copies start once it is ready
        from easydl_amd.utils.gshadow import HostShadow
        slot = f"{self.ctx.role}{self.ctx.index}"

        def make():
            t0 = time.perf_counter()
            try:
                hs = HostShadow(self.ctx.job, slot, self.flat.groups)
            except Exception as e:  # noqa: BLE001 - an optimisation: without it a step is recomputed
                self.events.emit("grad_shadow_failed", where="host", error=str(e)[:200])
                return
            self._hshadow_views = [(hs.group_views(i), hs.loss_view(i)) for i in (0, 1)]
            self._hshadow = hs
            self.events.emit("grad_shadow_ready", where="host", pinned=hs.pinned, gb=round(hs.total / 2**30, 1),
                             s=round(time.perf_counter() - t0, 3))
        threading.Thread(target=make, name="edl-gshadow", daemon=True).start()

    def _maybe_rehome(self) -> None:
        """Once a takeover's state is settled, move everything built on the dead worker's HBM into
        this process's own allocations, between two steps (FlatParams.rehome: one group at a
        time).  Imported memory cannot be exported again, so until then this process has
        nothing to hand to the next standby: a second failure of this rank would restore from
        /dev/shm instead of resuming from HBM.  Waits until the adopted state is verified (the
        post-reap step-mark check, an early hand-over's check, a deferred restore), full
        micro-batches are back and one group's copy fits in free HBM."""
        from easydl_amd.utils import vram
        if self._rehomed or not vram.adopted_any() or self.flat is None or self.opt is None:
            return
        if self.comm is None or self.comm.world_size > 1:
            # only one rank moves its buffers, and re-registering the moved gradients with the xGMI
            # engine is collective (a world-8 drill hung there); an HBM resume -- what the re-published
            # state is for -- happens at world 1 only, so the move waits for a world of one
            return
        ck = self.checkpoint
        if ck is not None and (getattr(ck, "_marks_check", None) is not None or getattr(ck, "_verify", None) is not None
                               or getattr(ck, "_deferred", None)):
            return
        if self._mb_split > 1 or self._mb_recompute is not None:
            return
        adopted = set(vram.TAKEN.values())
        before = {k: t for k, t in self.vram_state_tensors().items() if t.data_ptr() in adopted}
        sizes = [t.untyped_storage().nbytes() for t in before.values()]
        # weak references: which buffer still is the adopted one afterwards (a freed adopted
        # range's address can come back for a new allocation, so pointers cannot tell)
        before = {k: weakref.ref(t) for k, t in before.items()}
        refs = list(before.values())

        def is_adopted(t):
            return any(r() is t for r in refs)
        if self.device.type == "cuda" and sizes and self._hbm_avail() < 2 * max(sizes):
            return
        t0 = time.perf_counter()
        self.wait_update()
        if ck is not None:
            ck.wait()           # no snapshot copy may read a buffer while it moves
        if self.device.type == "cuda":
            # the new buffers get segments of their own (fresh allocations, not blocks split out
            # of a cached activation segment): an IPC export maps a buffer's whole segment
            torch.cuda.empty_cache()
        # each moved buffer frees its adopted original as the last reference goes; should one stay
        # referenced, HBM would shrink by a buffer per move: stop while the next step's
        # activations and two buffers still fit (the rest stays on adopted memory, still correct)
        reserve = getattr(self, "_act_need", 0) + 2 * max(sizes, default=0)
        can_continue = (lambda: self._hbm_avail() >= reserve) if self.device.type == "cuda" else (lambda: True)
        n = self._move_state(is_adopted, can_continue)
        left = [k for k, t in self.vram_state_tensors().items() if k in before and before[k]() is t]
        if self.device.type == "cuda":
            torch.cuda.current_stream(self.device).synchronize()
        self._rehomed = True    # (once: a partial move is not retried)
        if left:
            for k in [k for k in vram.TAKEN if k not in left]:
                vram.TAKEN.pop(k)
            self.events.emit("rehome_partial", buffers=n, left=left[:8], n_left=len(left), step=self.step,
                             avail_gb=round(self._hbm_avail() / 2**30, 1), s=round(time.perf_counter() - t0, 3))
            return
        vram.TAKEN.clear()
        vram.ADOPTED_FROM.clear()
        self.events.emit("rehomed", buffers=n, gb=round(sum(sizes) / 2**30, 2), step=self.step,
                         s=round(time.perf_counter() - t0, 3))
        self._publish_vram()    # the next standby can adopt this state again
        for attempt in range(5):
            # a buffer whose export failed ("invalid argument": 1-8 of 95 at Llama-3-8B, where a new
            # allocation reuses an address range an imported buffer had; profiles/r05_three_failures_8b.md) moves
            # once more, to another fresh allocation, and the state is published again
            if not vram.FAILED or self.device.type != "cuda":
                break
            names = list(vram.FAILED)
            ts = self.vram_state_tensors()
            targets = [ts[k] for k in names if k in ts]
            del ts
            self._move_state(lambda t: any(t is x for x in targets))
            del targets
            torch.cuda.current_stream(self.device).synchronize()
            self.events.emit("rehome_export_retry", names=names[:8], attempt=attempt + 1)
            self._publish_vram()

    def _move_state(self, pick, can_continue=lambda: True) -> int:
        """(World 1.) Move the state buffers ``pick(tensor)`` selects to fresh allocations of this process
        (FlatParams.rehome, optim.rehome_state, FlatBuffers.rehome).  Allocated from a private
        pool: every buffer gets a segment of its own, never a block of a cached (possibly
        > 2 GiB) segment, which fails to export."""
        from easydl_amd.optim import rehome_state
        alias = [st.get("master") is not None and st["master"].data_ptr() == g.data.data_ptr()
                 for g, st in zip(self.flat.groups, self.opt.state)]
        pool = torch.cuda.use_mem_pool(self._state_pool()) if self.device.type == "cuda" else _null()
        with pool:
            n = self.flat.rehome(pick, can_continue)
            for g, st, a in zip(self.flat.groups, self.opt.state, alias):
                if a:
                    st["master"] = g.data   # an fp32 model's master IS its weight buffer
            n += rehome_state(self.opt.state, pick, can_continue)
            if self.bufs is not None:
                n += self.bufs.rehome(pick, can_continue)
        if self.ddp is not None:
            self.ddp.set_bucket_mb(self.ddp.bucket_mb)      # bucket views of the new gradient buffers
        return n

    def _state_pool(self):
        if getattr(self, "_pool", None) is None:
            self._pool = torch.cuda.MemPool()
        return self._pool

    def _hbm_avail(self) -> int:
        free, _ = torch.cuda.mem_get_info(self.device)
        return free + torch.cuda.memory_reserved(self.device) - torch.cuda.memory_allocated(self.device)

    def _memory_plan(self) -> None:
        """A replacement that adopted a dead worker's HBM starts while the driver is still
        reclaiming the rest of that worker's memory (its activations: ~82 GB for Llama-3-8B at
        2 x 8k tokens per micro-batch).  A first step that needs more than the GPU has free
        blocks inside hipMalloc until the reclaim is done -- 6 s of an 8 s time-to-recover
        (profiles/r05_ttr_headline.md).  Instead, while memory is short, each micro-batch is
        split into smaller ones: the same samples, the same loss weights, the same gradient sum
        (only the order of the bf16 additions differs), at roughly half the activation memory.
        Models with dropout are the exception: the pieces of micro-batch i are seeded once and draw
        their masks one after another, so a split step is NOT bit-exact with the unsplit one there
        (Llama, the only model this path serves, has no dropout).
        When not even one sample per micro-batch fits, a model with a ``cfg.recompute`` switch
        (Llama) recomputes its layers' activations in the backward instead.
        Checked again before every step; full micro-batches return once the memory is back."""
        from easydl_amd.utils import vram
        self._mb_split = 1
        if self._mb_recompute is not None:
            self.model.cfg.recompute, self._mb_recompute = self._mb_recompute, None
        if (self.device.type != "cuda" or self.tp > 1 or not vram.adopted_any()
                or getattr(self, "kv", None) is None or os.environ.get("EDL_RECOVERY_SPLIT", "1") == "0"):
            return
        need, mbs = vram.read_act(self.kv, f"{self.ctx.role}{self.ctx.index}")
        if not need or mbs != self.micro_batch:
            return
        self._act_need = need
        avail = self._hbm_avail()
        if avail >= need * 1.05:
            return
        margin = float(os.environ.get("EDL_RECOVERY_MARGIN", "1.15"))
        k = next((d for d in range(2, mbs + 1) if mbs % d == 0 and need / d * margin <= avail), None)
        cfg = getattr(self.model, "cfg", None)
        if k is None and cfg is not None and isinstance(getattr(cfg, "recompute", None), bool):
            # even one sample per micro-batch would not fit: recompute each layer's activations in
            # the backward instead (same values, ~1/3 more compute) until the memory is back --
            # a step that blocks in hipMalloc behind the driver's reclaim costs seconds
            self._mb_recompute = cfg.recompute
            cfg.recompute = True
            k = 1
        self._mb_split = mbs if k is None else k
        self.events.emit("memory_limited_steps", split=self._mb_split, recompute=self._mb_recompute is not None,
                         need_gb=round(need / 2**30, 1), avail_gb=round(avail / 2**30, 1))

    def _split_micro_batches(self, mbs: list) -> list:
        if (self._mb_split > 1 or self._mb_recompute is not None) and self._hbm_avail() >= self._act_need * 1.05:
            self.events.emit("memory_restored", step=self.step, avail_gb=round(self._hbm_avail() / 2**30, 1))
            self._mb_split = 1
            if self._mb_recompute is not None:
                self.model.cfg.recompute, self._mb_recompute = self._mb_recompute, None
        k = self._mb_split
        if k <= 1:
            return mbs
        out = []
        for mb, idx in mbs:     # (micro-batch index, sample indices): the pieces keep the index
            idx = list(idx)
            n = -(-len(idx) // k)
            out += [(mb, idx[i:i + n]) for i in range(0, len(idx), n)]
        return out

    def _hbm_resume_step(self) -> int | None:
        """Step K if this process adopted a dead worker's HBM (utils/vram.py) whose step marks
        (utils/stepmarks.py) say the update of step K had finished and none was in flight."""
        from easydl_amd.utils import stepmarks, vram
        pid = vram.ADOPTED_FROM.get("pid")
        if (pid is None or self.tp > 1 or self.comm is None or self.comm.world_size != 1
                or os.environ.get("EDL_HBM_RESUME", "1") == "0"):
            return None
        marks = stepmarks.read_slot(self.ctx.job, f"{self.ctx.role}{self.ctx.index}", shadow=True)
        if marks is None:
            return None
        begin, done, writer, *shadow = marks
        self._shadow_cand = tuple(shadow)
        if writer != pid or begin != done:
            self.events.emit("hbm_resume_refused", begin=begin, done=done, writer=writer, adopted_from=pid)
            return None
        # every tensor of the training state must be the dead worker's: one that was not
        # exported, not mapped or not taken (size / dtype / layout changed) holds init values
        from easydl_amd.ckpt.manager import CheckpointManager
        need = CheckpointManager.state_of(self) + [(f"model.{g.name}", g.data) for g in self.flat.groups]
        miss = vram.missing(need)
        if miss:
            self.events.emit("hbm_resume_refused", reason="incomplete", missing=miss[:8], n_missing=len(miss),
                             of=len(need), begin=begin, done=done)
            return None
        return done

    def _maybe_restore(self, defer_moments: bool = False) -> bool:
        """State of a process that holds none: the dead worker's HBM (HBM resume), else the
        newest snapshot.  With neither, buffers adopted from a dead worker are reset to this
        process's seeded init (a fresh start).  True if trained state was recovered."""
        t0 = time.perf_counter()
        if self.checkpoint is not None:
            k = self._hbm_resume_step()
            if k is not None:
                from easydl_amd.utils import vram
                pid = vram.ADOPTED_FROM.get("pid")
                verify = None if vram.reaped(pid) else {"pid": pid, "marks": (k, k), "job": self.ctx.job,
                                                        "slot": f"{self.ctx.role}{self.ctx.index}"}
                from easydl_amd.utils.stepmarks import best_shadow
                cand = getattr(self, "_shadow_cand", (0, 0, 0, 0))
                sh = self.flat.shadow_tensors()
                host = not sh and self._host_shadow_exists()
                best = best_shadow(cand if host else cand[:2], k + 1)   # (the HBM shadow: slot 0 only)
                if (sh or host) and best is None and any(cand[1::2]):
                    self.events.emit("grad_shadow_unused", marks=list(cand), resume_step=k)
                if best is not None and (host or not vram.missing(list(sh.items()))):
                    # the dead worker had finished best[1] micro-batches of step k + 1 (their
                    # gradients are in its shadow): that step resumes there (_run_step)
                    self._shadow_resume = {"step": k + 1, "mb": best[1], "host": host, "slot": best[0]}
                    if verify is not None:
                        verify["shadow"] = tuple(cand)
                src = self.checkpoint.resume_from_hbm(self, k, verify)
                self.events.emit("restored", step=self.step, source=src, s=round(time.perf_counter() - t0, 3))
                return True
            st = self.checkpoint.restore_latest(self, defer_moments=defer_moments)
            if st is not None:
                from easydl_amd.ckpt import manager as _ckm
                self.events.emit("restored", step=self.step, source=st, s=round(time.perf_counter() - t0, 3),
                                 h2d=dict(_ckm.LAST_RESTORE_STATS))
                return True
        self._reinit_adopted()
        return False

    def _reinit_adopted(self) -> None:
        """Nothing overwrites this process's state: buffers it built on a dead worker's HBM
        (kept for an HBM resume that did not happen) go back to the seeded init."""
        from easydl_amd.utils import vram
        if not vram.adopted_any() or self.flat is None:
            return
        n = self.flat.reinit_adopted() + (self.bufs.reinit_adopted() if self.bufs is not None else 0)
        self.opt.reset_state()
        if self.device.type == "cuda":
            torch.cuda.current_stream(self.device).synchronize()
        self.events.emit("adopted_reinit", tensors=n)

    def _state_settled(self) -> None:
        if self.flat is not None:
            self.flat.drop_init_copies()
        if self.bufs is not None:
            self.bufs.drop_init_copies()

    # ------------------------------------------------------------------ steps
    def _micro_batches(self, data, plan: ElasticBatchPlan):
        c = self.dp_comm or self.comm  # TP ranks of one replica consume the same samples
        return plan.indices(self.step, c.rank, c.world_size)

    def _sync_buffers(self) -> None:
        """Module buffers (BatchNorm running statistics) are updated by each rank from its
        own micro-batches, so they drift apart; rank 0's copy is broadcast after every
        committed step (DDP's broadcast_buffers).  Snapshots shard the buffers like every
        other state tensor and assume all ranks hold the same bytes."""
        c = self.dp_comm
        if c is None or c.world_size == 1 or not self.bufs.tensors:
            return
        try:
            for t in self.bufs.tensors.values():
                c.broadcast(t, 0)
        except CommAborted:
            pass   # the epoch broke after the commit: the next epoch's state sync covers it

    def _seed_step(self, mb: int = 0) -> None:
        """Random streams keyed by (seed, committed step, data-parallel rank): dropout
        masks of step k do not depend on how the job got to step k (restarts, world
        changes), so a resume from a snapshot of step k replays step k+1 bit-exactly
        and a joiner taking over rank r draws what rank r would have drawn.  TP ranks
        of one replica share the stream (replicated activations need equal masks)."""
        c = self.dp_comm or self.comm
        r = c.rank if c is not None else 0
        torch.manual_seed((self._seed * 1_000_003 + self.step * 7_919 + r * 104_729 + mb * 15_485_863) % (1 << 62))

    def host_state(self) -> dict:
        """Host-side training state a resume needs besides the tensors (recorded in every
        snapshot and in the v1 manifest): the RNG policy + seed, the data-plan cursor and
        the LR schedule.  Steps and optimizer step count travel separately."""
        plan = getattr(self, "_plan", None)
        sched = getattr(self.opt, "schedule", None)
        return {"rng": {"policy": "per-step", "seed": self._seed},
                "data": {"cursor_step": self.step, "global_batch": self.global_batch,
                         "micro_batch": self.micro_batch, "plan_seed": getattr(plan, "seed", None),
                         "dataset_len": getattr(plan, "n", None)},
                "lr": sched.state_dict() if sched is not None else {"lr": getattr(self.opt, "lr", None)}}

    def load_host_state(self, h: dict | None) -> None:
        """Adopt a snapshot's host state (after its step has been restored)."""
        if not h:
            return
        self._seed = int(h.get("rng", {}).get("seed", self._seed))
        d = h.get("data", {})
        if d.get("global_batch") and self.global_batch and int(d["global_batch"]) != self.global_batch:
            log.warning("restored data plan had global batch %s, this run uses %s", d["global_batch"],
                        self.global_batch)
        lr = h.get("lr") or {}
        sched = getattr(self.opt, "schedule", None)
        if sched is not None and lr.get("total") is not None:
            sched.lr, sched.warmup, sched.total, sched.min_ratio = (lr["lr"], lr["warmup"], lr["total"],
                                                                    lr["min_ratio"])

    def _run_step(self, loss_fn, data, plan):
        mbs = list(enumerate(self._micro_batches(data, plan)))   # (micro-batch index, sample indices)
        self.flat.zero_grad()
        total = 0.0
        loss_acc = None
        if self._hshadow is not None and self._shadow_stream is not None:
            torch.cuda.current_stream(self.device).wait_stream(self._shadow_stream)
        res, self._shadow_resume = self._shadow_resume, None
        if res is not None and res["step"] == self.step + 1 and 0 < res["mb"] < len(mbs):
            # mid-step resume: the dead worker's gradients of micro-batches [0, mb) from its shadow
            if res.get("host"):
                loss_acc = self._load_host_shadow(res["slot"])
            else:
                self.flat.load_shadow()
                loss_acc = self.flat.gshadow_loss[0].clone()
            if loss_acc is not None:
                total = sum(len(idx) for _, idx in mbs[:res["mb"]]) / plan.global_batch
                self.events.emit("resumed_mid_step", step=self.step + 1, micro_batches_done=res["mb"],
                                 of=len(mbs), host=bool(res.get("host")))
                mbs = mbs[res["mb"]:]
        if self._mb_split > 1 or self._mb_recompute is not None:
            mbs = self._split_micro_batches(mbs)
        shadow = self._shadow_active()
        seeded = None
        with self.kmix.phase("compute"):
            for j, (i, idx) in enumerate(mbs):
                if self.comm is not None and self.comm.aborted:  # epoch broke: do not start more work
                    raise CommAborted(f"epoch {self.comm.epoch} aborted before micro-batch {i}")
                if i != seeded:
                    self._seed_step(i)      # random streams keyed by micro-batch: a mid-step resume replays them
                    seeded = i
                batch = data.batch(idx, self.device)
                w = len(idx) / plan.global_batch
                last = j == len(mbs) - 1
                ctxm = self.ddp.no_sync() if not last else _null()
                with ctxm, trace.range(f"microbatch{i}"):
                    with trace.range("fwd"):
                        loss = loss_fn(self.model, batch)
                    if self._shadow_pending:
                        # the shadow copy of the previous micro-batch's gradients must finish first
                        torch.cuda.current_stream(self.device).wait_stream(self._shadow_stream)
                        self._shadow_pending = False
                    with trace.range("bwd"):
                        (loss * w).backward() if w != 1.0 else loss.backward()
                ld = loss.detach() * w
                loss_acc = ld if loss_acc is None else loss_acc + ld
                total += w
                if shadow and not last:
                    self._shadow_grads(i + 1, loss_acc)
                if not last:
                    self.fault.maybe_inject("microbatch", self.step, trainer=self, mb=i)
        t_mb = time.perf_counter()
        if self._phases and self.device.type == "cuda":
            # diagnostic mode: drain the compute stream so 'finish' is the gradient all-reduce alone
            torch.cuda.current_stream(self.device).synchronize()
            self._t_host = t_mb - getattr(self, "_t_step", t_mb)
            t_mb = time.perf_counter()
        # a rank without samples (world > batch) still joins every all-reduce with zeros:
        # finish() zero-fills untouched gradients before flushing the buckets.
        with trace.range("grad_sync"):
            self.ddp.finish()
            if hasattr(self.model, "sync_sp_grads"):
                self.model.sync_sp_grads(self.flat)   # sequence-parallel norm grads: sum over TP
        self.fault.maybe_inject("after_backward", self.step, trainer=self)
        self._t_mb = t_mb
        return None if loss_acc is None else loss_acc / total

    def _host_shadow_exists(self) -> bool:
        from easydl_amd.utils.gshadow import seg_name
        return self.device.type == "cuda" and os.path.exists(
            "/dev/shm" + seg_name(self.ctx.job, f"{self.ctx.role}{self.ctx.index}"))

    def _opt_overlap(self):
        """The optimizer stream when the update may overlap the next step's forward, else None.

        The update of 8B parameters is ~42 ms a step of memory-bound kernels (AdamW reads and
        writes 30 B per parameter) that the compute-bound forward GEMMs leave bandwidth for.  So
        the update runs on a side stream, group by group in the order the next forward reads the
        groups.  Every module waits only for its own parameters' group before its forward
        (FlatParams install_update_waits; Llama awaits its embedding and head itself), and every
        gradient write waits for the update that still reads that gradient (gradsink
        await_shadow).  Off for models with module buffers (BatchNorm statistics are broadcast
        after the update), tensor parallelism, optimizers without per-group callbacks, and with
        ``EDL_OPT_OVERLAP=0``.  An ``on_step`` callback runs while the update may still be in
        flight: one that reads parameters directly calls ``wait_update()`` first."""
        if self._opt_stream is not None:
            return self._opt_stream
        if self._opt_overlap_off:
            return None
        if (self.device.type != "cuda" or self.tp > 1 or os.environ.get("EDL_OPT_OVERLAP", "1") == "0"
                or not getattr(self.opt, "supports_group_done", False)
                or (self.bufs is not None and self.bufs.tensors)):
            self._opt_overlap_off = True
            return None
        from easydl_amd.ops import fused
        from easydl_amd.parallel.flat import install_update_waits
        install_update_waits(self.model)
        fused._WT_BATCH = False     # the batched W^T refresh would read every weight at the first use
        self._opt_stream = torch.cuda.Stream(device=self.device)
        self._opt_stream.wait_stream(torch.cuda.current_stream(self.device))
        return self._opt_stream

    def _order_update_after_step(self, ovl) -> None:
        """The update of step k reads step k's gradients and rewrites the weights its backward
        read for dgrad: it starts after everything the compute stream holds at the commit (every
        micro-batch's backward, the fused ops' side-stream weight gradients, which ddp.finish
        joined into it, and finalize_untouched).  Every step, not once at stream creation: at
        world 1 the host does not drain the step (_sync_point), so without this edge the update
        could run while the backward still writes the gradients it reads."""
        ovl.wait_stream(torch.cuda.current_stream(self.device))

    def _opt_group_done(self, i: int) -> None:
        ev = torch.cuda.Event()
        ev.record(self._opt_stream)
        for sl in self.flat.groups[i].slots:
            sl.param._edl_fwd_wait = ev      # its next reader waits for this group's update
            sl.param._edl_wait = ev          # its next gradient write waits for the update's read

    def wait_update(self) -> None:
        """Order the current stream after the last optimizer update (see _opt_overlap)."""
        if self._opt_stream is not None:
            torch.cuda.current_stream(self.device).wait_stream(self._opt_stream)

    def _shadow_wanted(self) -> bool:
        """Gradient shadows pay off where a replacement resumes from this process's HBM: one rank
        (HBM resume needs world 1), VRAM hand-over on, several micro-batches per step."""
        from easydl_amd.utils import vram
        return (vram.enabled() and self.device.type == "cuda" and self.tp == 1 and self.flat is not None
                and self.comm is not None and self.comm.world_size == 1 and self.global_batch is not None
                and self.global_batch > self.micro_batch and os.environ.get("EDL_GRAD_SHADOW", "1") != "0")

    def _shadow_active(self) -> bool:
        return (self._marks is not None and (self.flat.gshadow is not None or self._hshadow is not None)
                and self._mb_split == 1 and self.comm.world_size == 1)

    def _shadow_grads(self, mbs_done: int, loss_acc) -> None:
        """After a micro-batch's backward: copy the accumulated gradients (and the partial loss)
        into the shadow on a side stream, under the next micro-batch's forward, between an
        invalidating and a validating step mark (utils/stepmarks.py).  The next backward waits
        for the copy.  Gradients no micro-batch has written yet are zeroed first (as the end of
        the step would), so the shadow is exact."""
        self.flat.finalize_untouched()
        if self.flat.gshadow is None:
            self._shadow_to_host(mbs_done, loss_acc)
            return

        def copy(st):
            self._marks.shadow(self.step + 1, 0, st)
            with torch.no_grad():
                for g, t in zip(self.flat.groups, self.flat.gshadow):
                    t.copy_(g.grad)
                self.flat.gshadow_loss.copy_(loss_acc.reshape(1))
            self._marks.shadow(self.step + 1, mbs_done, st)
        if self.device.type != "cuda":
            copy(None)
            return
        if self._shadow_stream is None:
            self._shadow_stream = torch.cuda.Stream(device=self.device)
        st = self._shadow_stream
        st.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(st):
            copy(st)
        loss_acc.record_stream(st)
        self._shadow_pending = True

    def _load_host_shadow(self, slot: int):
        """The dead worker's host shadow ``slot`` -> this process's gradient buffers (pipelined
        shm -> HBM copy); returns the partial loss (a 0-d CUDA tensor), None if it failed."""
        from easydl_amd.utils.gshadow import HostShadow
        t0 = time.perf_counter()
        loss = torch.zeros(1, dtype=torch.float32, device=self.device)
        stats: dict = {}
        try:
            hs = HostShadow(self.ctx.job, f"{self.ctx.role}{self.ctx.index}", self.flat.groups, create=False,
                            pin=False)
            try:
                hs.load_into(self.flat.groups, loss, slot, stats)
            finally:
                hs.close()
        except (OSError, RuntimeError) as e:
            # the whole step is recomputed instead, from zeroed gradients (a failed copy may have
            # written part of them)
            with torch.no_grad():
                for g in self.flat.groups:
                    g.grad.zero_()
            self.events.emit("grad_shadow_load_failed", where="host", error=str(e)[:200])
            return None
        self.flat.mark_accumulating()
        self.events.emit("grad_shadow_loaded", where="host", slot=slot, s=round(time.perf_counter() - t0, 3),
                         gbps=stats.get("gbps"))
        return loss[0]

    def _shadow_to_host(self, mbs_done: int, loss_acc) -> None:
        """Host gradient shadow (utils/gshadow.py): device -> host copies group by group on a side
        stream, in the order the next backward writes the groups; each parameter's next write
        waits for its group's copy only (gradsink.await_shadow), not the next micro-batch for all
        of them."""
        slot = self._hshadow_next = 1 - getattr(self, "_hshadow_next", 1)   # alternate: 0, 1, 0, ...
        views, loss_view = self._hshadow_views[slot]
        main = torch.cuda.current_stream(self.device)
        if self._shadow_stream is None:
            self._shadow_stream = torch.cuda.Stream(device=self.device)
        st = self._shadow_stream
        st.wait_stream(main)
        with torch.cuda.stream(st):
            self._marks.shadow(self.step + 1, 0, st, slot)
            for g, hv in zip(self.flat.groups, views):
                hv.copy_(g.grad.view(-1), non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(st)
                for sl in g.slots:
                    sl.param._edl_wait = ev
            loss_view.copy_(loss_acc.reshape(1).float(), non_blocking=True)
            self._marks.shadow(self.step + 1, mbs_done, st, slot)
        loss_acc.record_stream(st)

    def _sync_point(self) -> bool:
        """Host-side completion of every gradient all-reduce; False if the epoch broke.

        At world 1 there is no collective whose outcome the commit must wait for, so the
        host does not drain the stream: it goes on enqueueing the optimizer and the next
        step while the GPU works (no per-step bubble; EDL_STEP_SYNC=1 restores the drain)."""
        if self.device.type == "cuda" and (self.comm.world_size > 1 or self._step_sync or self._sync_next):
            # (the first step of an epoch always completes on the GPU before it counts:
            # time-to-recover is measured to a finished step)
            torch.cuda.current_stream(self.device).synchronize()
        self._sync_next = False
        if self.comm.aborted:
            return False
        if not self.comm.healthy():  # a hand-written collective hit its deadline: the grads are not a sum
            log.warning("epoch %d: a bounded collective gave up; dropping step %d", self.comm.epoch, self.step)
            self.comm.abort()
            return False
        return True

    def fit(self, loss_fn, data, num_steps: int, on_step=None) -> "ElasticTrainer":
        """Train until ``num_steps`` committed steps.  ``loss_fn(model, batch) -> scalar loss``."""
        gb = self.global_batch
        if gb is None:
            w = self.ctx.static_world or 1
            gb = w * self.micro_batch
            self.global_batch = gb
        plan = ElasticBatchPlan(len(data), gb, self.micro_batch, seed=17)
        self._plan = plan
        if os.environ.get("EDL_PREJOIN_WARMUP", "1") != "0":
            self._prejoin = lambda: self._prejoin_warmup(loss_fn, data, plan)
        self._connect()
        self._start_watchdog()
        try:
            try:
                self._enter_epoch()
            except JobFinished:
                self.events.emit("finished_waiting", node=self.ctx.node_id)
                return self
            self._publish_vram()
            self._open_marks()
            self._publish_warm_spec(data)
            prof = None
            if os.environ.get("EDL_PROFILE_FIRST_STEP", "0") == "1":
                import cProfile         # diagnostics: host profile of this process's first step
                prof = cProfile.Profile()
                prof.enable()
            while self.step < num_steps and not self._stop_requested:
                if prof is not None and self.history:
                    prof.disable()
                    self._dump_profile(prof)
                    prof = None
                t0 = self._t_step = time.perf_counter()
                ok = True
                loss = None
                try:
                    self.fault.maybe_inject("step_start", self.step, trainer=self)
                    loss = self._run_step(loss_fn, data, plan)
                    t_run = time.perf_counter()
                    ok = self._sync_point()
                    t_sync = time.perf_counter()
                except CommAborted as e:
                    log.warning("step %d aborted: %s", self.step, e)
                    ok = False
                except RuntimeError as e:
                    if self.comm is not None and (self.comm.aborted or _is_comm_error(e)):
                        log.warning("step %d failed in communication: %s", self.step, e)
                        ok = False
                    else:
                        raise
                if self._master_lost is not None:
                    raise MasterUnreachable(f"job master unreachable: {self._master_lost}")
                if self.rdzv is not None:
                    apply, latest = self.rdzv.commit(self.comm.epoch, self.step, self.comm.world_size, ok,
                                                     gc=self.comm.rank == 0)
                else:
                    apply, latest = ok, 0
                t_commit = time.perf_counter()
                if apply:
                    ovl = self._opt_overlap()
                    if ovl is not None:
                        self._order_update_after_step(ovl)
                    upd = _null() if ovl is None else torch.cuda.stream(ovl)
                    with upd:   # (overlap: the update runs on its own stream under the next forward)
                        if self.checkpoint is not None:
                            self.checkpoint.fence()  # never update params under an in-flight snapshot
                            hv = self.checkpoint.stats.pop("handover_verified_s", None)
                            if hv is not None:
                                self.events.emit("handover_verified", step=self.step, s=hv)
                                self._open_marks()
                        t_fence = time.perf_counter()
                        if self._marks is not None:
                            self._marks.begin(self.step + 1, torch.cuda.current_stream(self.device)
                                              if self.device.type == "cuda" else None)
                        with trace.range("optimizer"), self.kmix.phase("memory"):
                            if ovl is None:
                                self.opt.step(pre_scale=1.0)
                            else:
                                self.opt.step(pre_scale=1.0, group_done=self._opt_group_done)
                        self.fault.maybe_inject("in_update", self.step, trainer=self)
                        self._sync_buffers()
                        if self._marks is not None:
                            self._marks.done(self.step + 1, torch.cuda.current_stream(self.device)
                                             if self.device.type == "cuda" else None)
                    if self._phases and ok:
                        # host-side split of one step (EDL_STEP_PHASES=1): enqueue of the micro-batches,
                        # wait for the GPU (compute + all-reduce), commit round, snapshot fence, optimizer
                        self.events.emit("step_phases", step=self.step + 1, run=round(t_run - t0, 4),
                                         mb=round(self._t_mb - t0, 4), finish=round(t_run - self._t_mb, 4),
                                         mb_host=round(getattr(self, "_t_host", 0.0), 4),
                                         sync=round(t_sync - t_run, 4), commit=round(t_commit - t_sync, 4),
                                         fence=round(t_fence - t_commit, 4),
                                         opt=round(time.perf_counter() - t_fence, 4))
                    self.step += 1
                    self.last_loss = loss
                    rec = {"step": self.step, "epoch": self.comm.epoch, "world": self.comm.world_size,
                           "dt": time.perf_counter() - t0}
                    self.history.append(rec)
                    self.events.emit("step_done", step=self.step, epoch=self.comm.epoch,
                                     world=self.comm.world_size)
                    self.metrics.record(self.step, rec["dt"], samples=self.global_batch,
                                        tokens=self.global_batch * self.tokens_per_sample, world=self.comm.world_size,
                                        loss=None, extra=self._metrics_extra)
                    if self.checkpoint is not None:
                        with upd:       # a snapshot copies the state after the update
                            self.checkpoint.on_step(self)
                    if latest > self.comm.epoch:
                        # the agreed decision already names a newer epoch (a rejoin, a scale-up):
                        # a probe of THIS world would be thrown away, and would hold the rejoin
                        # back by its length (8 s with 7 ranks time-slicing one GPU,
                        # profiles/r05_world8_shared_gpu.md).  Every rank read the same decision.
                        self._skip_deferred_probes(latest)
                    else:
                        self._run_deferred_probes()
                    self._publish_act()
                    self._maybe_rehome()
                    if on_step is not None:
                        on_step(self, loss)
                    if self.log_every and self.step % self.log_every == 0 and self.comm.rank == 0:
                        log.info("step %d loss %.4f world %d", self.step, float(loss), self.comm.world_size)
                else:
                    self.events.emit("step_dropped", step=self.step, epoch=self.comm.epoch)
                if self.rdzv is not None and self.rdzv.plan_version != self.plan_version:
                    self._apply_runtime_plan(self.rdzv.plan_version)
                need_new = (not ok) or self.comm.aborted or (self.rdzv is not None and latest > self.comm.epoch)
                if need_new and self.step < num_steps and not self._stop_requested:
                    try:
                        self._reconfigure()
                    except JobFinished:
                        self.events.emit("finished_waiting", node=self.ctx.node_id)
                        return self
            if self.rdzv is not None and self.comm.rank == 0:
                self.rdzv.kv.set("train/done", str(self.step))  # releases spare waiting workers
        finally:
            self._stop.set()
            if self.device.type == "cuda":
                self.wait_update()      # the caller reads the trained state next
        return self

    def _metrics_extra(self) -> dict:
        from easydl_amd.utils.metrics import cu_count
        return {"role": self.ctx.role, "gpu_mix": self.kmix.snapshot(), "cu": cu_count(self.ctx.cu_mask),
                "device": self.device.type}

    def _dump_profile(self, prof) -> None:
        import io
        import pstats
        out = io.StringIO()
        st = pstats.Stats(prof, stream=out)
        st.sort_stats("cumulative").print_stats(40)
        st.sort_stats("tottime").print_stats(25)
        log.warning("first-step host profile (step %d):\n%s", self.step, out.getvalue())
        print(out.getvalue(), file=__import__("sys").stderr, flush=True)

    def _skip_deferred_probes(self, latest: int) -> None:
        for group, c in self._comm_groups():
            if getattr(c, "probe_pending", False):
                self.events.emit("allreduce_probe_skipped", epoch=self.comm.epoch, group=group, step=self.step,
                                 next_epoch=latest)

    def _run_deferred_probes(self) -> None:
        """A re-formed epoch's all-reduce probe, deferred off the recovery path: run after
        its first committed step (every rank reaches this point after the same commit).
        A failure here breaks the epoch like any collective failure."""
        ran = False
        for group, c in self._comm_groups():
            if not getattr(c, "probe_pending", False):
                continue
            try:
                s = c.run_deferred_probe()
            except (CommAborted, RuntimeError) as e:
                if not (c.aborted or _is_comm_error(e)):
                    raise
                log.warning("deferred all-reduce probe failed: %s", e)
                self.comm.abort()
                return
            ran = True
            self.events.emit("allreduce_probe_deferred", epoch=self.comm.epoch, group=group, step=self.step,
                             s=round(s, 4), selected=(c.xgmi_probe or {}).get("selected"))
        if ran:
            if self.rdzv is not None:
                self._publish_probe()
            if getattr(self.dp_comm, "xgmi", None) is not None:
                self.ddp.set_comm(self.dp_comm)   # map the gradient buffers for the engine

    def _apply_runtime_plan(self, version: int) -> None:
        """Brain runtime knobs of plan ``version`` (master/planner.py writes one document
        per version), switched by every rank at the same committed step or epoch entry."""
        self.plan_version = version
        doc = self.kv.get(f"plan/runtime/{version}")
        if not isinstance(doc, dict):
            return
        mb = doc.get("bucket_mb")
        if mb and float(mb) != self.ddp.bucket_mb:
            self.ddp.set_bucket_mb(float(mb))
            self.events.emit("plan_bucket_mb", mb=float(mb), step=self.step)
        ci = doc.get("ckpt_interval")
        if ci and self.checkpoint is not None:
            self.checkpoint.interval = max(1, int(ci))
        if doc.get("warm_window"):
            self._warm_window(doc["warm_window"])
        for group, c in self._comm_groups():
            ar = (doc.get("allreduce") or {}).get(group)
            apply = getattr(c, "adopt_policy", None) or getattr(c, "apply_allreduce_policy", None)
            if ar and apply is not None and int(ar.get("world", -1)) == c.world_size and apply(ar["policy"]):
                self.events.emit("plan_allreduce", step=self.step, group=group, world=ar["world"],
                                 policy=ar["policy"])
                if c is self.dp_comm and self.ddp is not None and getattr(c, "xgmi", None) is not None:
                    self.ddp.set_comm(c)   # the engine may have just been switched on: map the buffers

    def _reconfigure(self):
        old = self.comm
        self.events.emit("reconfigure", epoch=old.epoch, aborted=old.aborted)
        if old.aborted:
            pass
        else:
            old.shutdown()
        _retire(old, self.events)
        del old
        if self.rdzv is not None and self.rdzv.kv.exists(f"rdzv/leave/{self.ctx.node_id}"):
            raise SystemExit(0)
        self._enter_epoch()
        self._settle_marks()

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


class MasterUnreachable(RuntimeError):
    """The job master's store stopped answering (see ElasticTrainer._start_watchdog)."""


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


_RELEASES: list[threading.Thread] = []   # aborted engines being released (_retire)


def _join_releases(timeout_s: float = 10.0) -> None:
    """Wait for the aborted engines' releases before a new engine allocates and exports its
    workspace: a workspace exported (hipIpcGetMemHandle) while the old one is being freed on
    another thread failed with hipErrorInvalidValue in a 4-rank kill drill (batch 30).  The
    release is quick -- the abort word ends every spin -- (2-40 ms measured)."""
    t_end = time.monotonic() + timeout_s
    while _RELEASES:
        th = _RELEASES[0]
        th.join(max(0.0, t_end - time.monotonic()))
        if th.is_alive():
            log.warning("an aborted xGMI engine is still being released; building the next one anyway")
            return
        _RELEASES.pop(0)


def _retire(comm, events=None) -> None:
    """Shorten the teardown of an aborted epoch's gloo groups.  A ProcessGroupGloo whose
    collective was abandoned on a dead peer blocks in its destructor until that collective
    times out; two survivors dropping their old groups at once can each wait for the other's
    sockets for the full timeout (~120 s measured: the new epoch's first step stalled).  The
    groups get a short timeout first, so the abandoned collective fails within seconds."""
    if not getattr(comm, "aborted", False):
        return
    x = getattr(comm, "xgmi", None)
    if x is not None and hasattr(x, "close_after_abort"):
        # The aborted epoch's engine still maps its peers' registered buffers (a dead peer's
        # included: the mapping keeps that HBM allocated) and owns a workspace; release them
        # off the recovery path once its stream has drained (the abort word ends every spin).
        comm.xgmi = None

        def _release(eng=x, epoch=getattr(comm, "epoch", None)):
            t0 = time.perf_counter()
            try:
                eng.close_after_abort()
            except Exception as e:  # noqa: BLE001
                log.warning("releasing an aborted xGMI engine failed: %s", e)
            if events is not None:
                events.emit("xgmi_released", epoch=epoch, s=round(time.perf_counter() - t0, 3))
        th = threading.Thread(target=_release, name="edl-xgmi-release", daemon=True)
        _RELEASES.append(th)
        th.start()
    import datetime
    for pg in (getattr(comm, "data", None), getattr(comm, "ctrl", None)):
        if isinstance(pg, dist.ProcessGroupGloo):
            try:
                pg.set_timeout(datetime.timedelta(seconds=2))
            except Exception:  # noqa: BLE001 - best effort
                pass


def _is_comm_error(e: Exception) -> bool:
    from easydl_amd.parallel.errors import is_comm_error
    return is_comm_error(e)
