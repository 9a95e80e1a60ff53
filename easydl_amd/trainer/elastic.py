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
from easydl_amd.trainer.recovery import RecoveryMixin, _null
from easydl_amd.utils import fault, trace
from easydl_amd.utils.events import EventLog
from easydl_amd.utils.metrics import MetricsReporter
from easydl_amd.utils.resources import apply_plan

log = logging.getLogger(__name__)

# Our watchdog decides when to abort RCCL; the PG must not crash the process itself.
os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "0")


class ElasticTrainer(RecoveryMixin):
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
        self._mb_limited = False     # a takeover's steps run short of HBM: re-planned per micro-batch
        self._mb_plan = (1, 0)       # (split, recomputed layers) in force
        self._shadow_stream = None   # gradient shadow copies (_shadow_grads)
        self._shadow_pending = False
        self._shadow_resume = None   # {"step", "mb", "host"}: resume that step at that micro-batch
        self._hshadow = None         # host gradient shadow (utils/gshadow.py), when HBM has no room
        self._opt_stream = None      # optimizer update overlapping the next forward (_opt_overlap)
        self._opt_overlap_off = False
        self._act_need = 0
        self._step_ev = None         # GPU event at the current step's start (fault after_ms counts from it)
        self._gpu_step_evs = []      # (step, start event) not yet paired: GPU step durations
        self._gpu_last = None        # (step, seconds) newest GPU-timed step
        self._snap_steps: set = set()   # steps whose update waited for a snapshot copy (GPU step clock)

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
        shadow = self._shadow_active()
        seeded = None
        probe = self.kmix.probe_due(self.step) and not self._mb_limited and self.tp == 1
        with self.kmix.phase("compute", probe=probe):   # (probe: on half the CUs, utils/kmix.py)
            ptrace = self._piece_trace_begin()
            for i, idx, last in self._pieces(mbs):   # (a memory-limited step: pieces, recompute)
                if self.comm is not None and self.comm.aborted:  # epoch broke: do not start more work
                    raise CommAborted(f"epoch {self.comm.epoch} aborted before micro-batch {i}")
                if ptrace is not None:
                    self._piece_trace_mark(ptrace, i, len(idx))
                if i != seeded:
                    self._seed_step(i)      # random streams keyed by micro-batch: a mid-step resume replays them
                    seeded = i
                batch = data.batch(idx, self.device)
                w = len(idx) / plan.global_batch
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
            if ptrace is not None:
                self._piece_trace_mark(ptrace, None, 0)
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

    _OVERLAP_MIN_GROUPS = 4

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
        flight: one that reads parameters directly calls ``wait_update()`` first.

        Default ("auto"): only for models of at least ``_OVERLAP_MIN_GROUPS`` flat groups (each
        <= 1.9 GB of gradients): with one or two groups the next forward waits for the whole
        update anyway, and the per-module wait hooks cost host time a short step cannot hide --
        BERT-large (1 group, 46 ms steps) ran 662 vs 700 samples/s with it on; Llama-3-8B
        (9 groups) 23,677 vs 23,649 tok/s (profiles/r06_opt_overlap_ab.jsonl,
        r06_bert_groups.jsonl).  ``EDL_OPT_OVERLAP=1`` forces it on."""
        if self._opt_stream is not None:
            return self._opt_stream
        if self._opt_overlap_off:
            return None
        mode = os.environ.get("EDL_OPT_OVERLAP", "auto")
        if (self.device.type != "cuda" or self.tp > 1 or mode == "0"
                or (mode != "1" and (self.flat is None or len(self.flat.groups) < self._OVERLAP_MIN_GROUPS))
                or not getattr(self.opt, "supports_group_done", False)
                or (self.bufs is not None and self.bufs.tensors)):
            self._opt_overlap_off = True
            return None
        from easydl_amd.ops import fused
        from easydl_amd.parallel.flat import install_update_waits
        install_update_waits(self.model)
        fused._WT_BATCH = False     # the batched W^T refresh would read every weight at the first use
        from easydl_amd.utils.resources import new_stream
        self._opt_stream = new_stream(self.device)     # CU-masked under a Brain CU plan
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
                self._mark_gpu_step_start()
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
                        self._mark_gpu_step_end()   # (on the update's stream)
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
                                     world=self.comm.world_size, dt=round(rec["dt"], 4), **self._gpu_step_time())
                    if self.checkpoint is not None and self.step % max(1, int(getattr(self.checkpoint, "interval", 0)
                                                                            or 1)) == 0:
                        self._snap_steps.add(self.step + 1)   # its update waits for this snapshot's copy
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
                    self._piece_trace_emit()
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

    def _mark_gpu_step_start(self) -> None:
        """Record a GPU event where this step starts on the compute stream.  At world 1 the host
        runs ahead of the GPU (no per-step drain, _sync_point), so host timestamps are enqueue
        times; GPU step durations and the fault injector's ``after_ms`` (utils/fault.py) use
        these events instead."""
        if self.device.type != "cuda":
            return
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(torch.cuda.current_stream(self.device))
        self._step_ev = ev
        self._gpu_step_evs.append([self.step, ev, None])
        del self._gpu_step_evs[:-64]

    def _mark_gpu_step_end(self) -> None:
        """The step's update is enqueued (current stream: the update's): its end event.  A GPU
        step = start of its forward -> end of its update, read without blocking once both have
        completed -- idle gaps BETWEEN steps (a host busy pinning snapshot memory) do not count."""
        if self.device.type != "cuda" or not self._gpu_step_evs or self._gpu_step_evs[-1][2] is not None:
            return
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(torch.cuda.current_stream(self.device))
        self._gpu_step_evs[-1][2] = ev
        q = self._gpu_step_evs
        # both events: start and end sit on different streams (compute / update), so an end
        # can complete first when the update is not ordered after the step
        while q and q[0][2] is not None and q[0][2].query() and q[0][1].query():
            s0, e0, e1 = q.pop(0)
            self._gpu_last = (s0 + 1, e0.elapsed_time(e1) / 1000.0)
        while q and q[0][2] is None and len(q) > 1:    # a dropped step: no end event
            q.pop(0)

    def _gpu_step_time(self) -> dict:
        """Newest completed GPU step duration for the step_done event (empty on the CPU); a step
        whose update waited for an in-memory snapshot's copy is flagged."""
        if self._gpu_last is None:
            return {}
        k = self._gpu_last[0]
        out = {"gpu_step": k, "gpu_s": round(self._gpu_last[1], 5)}
        if k in self._snap_steps:
            out["gpu_after_snapshot"] = True
        return out

    def _metrics_extra(self) -> dict:
        from easydl_amd.utils.metrics import cu_count
        out = {"role": self.ctx.role, "gpu_mix": self.kmix.snapshot(), "cu": cu_count(self.ctx.cu_mask),
               "device": self.device.type}
        if self.device.type == "cuda":
            # the Brain's per-rank HBM plan: what this rank's allocator actually holds at its peak
            out.update(gpu=self.device.index, hbm_peak_gb=round(torch.cuda.max_memory_reserved(self.device) / 2**30, 2),
                       hbm_total_gb=round(torch.cuda.get_device_properties(self.device).total_memory / 2**30, 1),
                       hbm_cap_gb=self.ctx.hbm_gb)
        return out

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
        if doc.get("cu_probe"):
            self.kmix.request_probe()     # the Brain wants a fresh CU-sensitivity measurement
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
