"""ElasticOperator re-cast as a local process manager for the GPUs of one node
(BASELINE.json north star; reference README.md:12 and
docs/design/elastic-training-operator.md:3-4,47-55,97-114).

Reference semantics kept:
* on ElasticJob submission ONLY the trainer (job master) is created (:47,105);
* the trainer queries the Brain, generates and applies a JobResource (:106-108);
* on JobResource create/update the operator creates / removes role processes
  to match ``replicas`` (:52-55,108-114) — horizontal scaling;
* ``resource_updation: [{name, resource}]`` launches a new process with the new
  resource that replaces the named one (:99-101) — vertical scaling;
* processes are named ``<job>-<role>-<index>`` (:87,91).

Local re-cast: "pods" are processes spawned by the native supervisor
(csrc/runtime/supervisor.cpp) with one GPU each (``EDL_GPU``), CPU affinity
and the plan's CU/HBM limits in the environment.  Exit events are forwarded to
the job master's store (``ev/exit/<node>``) the moment they happen, which is
what makes worker-death detection sub-millisecond.  Failed workers are
replaced (same name, new incarnation); clean exits mark completion.
"""
from __future__ import annotations

import json
import logging
import os
import shlex
import signal
import socket
import sys
import time
from dataclasses import dataclass, field

from easydl_amd.api.spec import ROLE_SHORT, ElasticJob, JobResource, Resource
from easydl_amd.utils.events import EventLog
from easydl_amd.utils.procfs import exit_status, mm_released

log = logging.getLogger("edl.operator")

REPO_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


@dataclass
class Proc:
    name: str
    role: str           # long role name (worker / parameter_server / evaluator / trainer)
    index: int
    pid: int
    gpu: int | None
    resource: Resource
    started: float
    state: str = "running"   # running | leaving | exited | completed | replaced
    exit_code: int | None = None
    generation: int = 0

    @property
    def node_id(self) -> str:
        return f"{self.name}:{self.pid}"


@dataclass
class OperatorConfig:
    gpus: list[int] = field(default_factory=list)       # GPU ordinals to hand out (repeat = shared slots)
    cpus: list[int] = field(default_factory=list)       # host CPUs to partition (affinity)
    max_restarts: int = 100
    leave_grace_s: float = 30.0
    master_port: int | None = None
    python: str = sys.executable
    replace_failed: bool = True
    standby: int = 0            # warm spare processes for the worker role (easydl_amd/operator/standby.py)


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def cu_mask_hex(n_cu: int, total: int = 256, start: int = 0) -> str:
    """Mask string for ``n_cu`` CUs; spread evenly over the 8 XCDs when possible."""
    n_cu = max(1, min(total, int(n_cu)))
    bits = 0
    per_xcd = total // 8
    take = [n_cu // 8 + (1 if x < n_cu % 8 else 0) for x in range(8)]
    for x in range(8):
        for c in range(take[x]):
            # hardware CU numbering interleaves XCDs: cu id = c * 8 + xcd
            bits |= 1 << ((start + c) % per_xcd * 8 + x)
    return hex(bits)


def hw_queues_capped(gpus: list, standbys: int, per_gpu_queues: int = 8) -> bool:
    """Whether the job's processes must run with fewer hardware queues each.

    Every process holds HIP's default of 4 hardware queues on each GPU it touches.  A standby
    touches EVERY GPU of the node (it imports each worker's exported HBM and warms up on each),
    and a rank's GPU may be shared by several ranks; the contexts on the busiest GPU are
    therefore ``max ranks per GPU + standbys``.  Past ``per_gpu_queues`` (8: a worker and one
    standby at 4 each, the N=8 layout) the cap applies to all of them -- standbys included,
    since they run the replacement in-process."""
    counts: dict = {}
    for g in gpus:
        counts[g] = counts.get(g, 0) + 1
    busiest = max(counts.values(), default=1)
    return busiest > 1 or (busiest + max(0, int(standbys))) * 4 > per_gpu_queues


class ElasticOperator:
    def __init__(self, job: ElasticJob, run_dir: str, launcher=None, cfg: OperatorConfig | None = None,
                 job_resource: JobResource | None = None, master_argv: list[str] | None = None, kv=None):
        self.job = job
        self.run_dir = os.path.abspath(run_dir)
        os.makedirs(self.run_dir, exist_ok=True)
        self.cfg = cfg or OperatorConfig()
        if launcher is None:
            from easydl_amd.operator.supervisor import Supervisor
            launcher = Supervisor()
        self.launcher = launcher
        self.events = EventLog(os.path.join(self.run_dir, "events-operator.jsonl"), proc="operator")
        self.procs: dict[str, Proc] = {}          # name -> current incarnation
        self.history: list[Proc] = []
        self.restarts = 0
        self.desired: JobResource | None = job_resource
        self.applied_version = -1
        self.applied_updations: set[tuple[int, str]] = set()
        self.master_port = self.cfg.master_port or free_port()
        self.master_argv = master_argv
        self.kv = kv
        self.overrides: dict[str, Resource] = {}
        self.done = False
        self.failed = False
        self._free_gpus = list(self.cfg.gpus)
        self.standbys: dict[str, Proc] = {}      # name -> parked spare
        self._ready_seen: set[str] = set()
        self._roster = None
        self._standby_seq = 0
        self._last_takeover = 0.0

    # ------------------------------------------------------------- master
    def start(self) -> None:
        """Create ONLY the trainer (job master) process first (reference :47,105-106)."""
        if os.environ.get("EDL_KEEP_SEGMENTS", "0") != "1":
            # the operator owns the job's /dev/shm segments (snapshots, PS shards, step marks):
            # a new job of the same name must not restore a previous run's state
            from easydl_amd.ckpt.manager import unlink_job_segments
            n = unlink_job_segments(self.job.name)
            if n:
                self.events.emit("stale_segments_removed", n=n)
        with open(os.path.join(self.run_dir, "job.json"), "w") as f:
            json.dump(self.job.to_dict(), f)
        argv = self.master_argv or [self.cfg.python, "-m", "easydl_amd.master.main", "--job", self.job.name,
                                    "--port", str(self.master_port), "--run-dir", self.run_dir,
                                    "--min", str(self.job.min_workers), "--max", str(self.job.max_workers),
                                    "--initial", str(self.desired.replicas("worker") if self.desired else 0),
                                    "--job-spec", os.path.join(self.run_dir, "job.json")]
        if self.desired is not None and self.master_argv is None:
            # a user-supplied JobResource is handed to the master, which applies it
            # instead of consulting the Brain
            jr_path = os.path.join(self.run_dir, "jobresource.json")
            with open(jr_path, "w") as f:
                json.dump(self.desired.to_dict(), f)
            argv += ["--job-resource", jr_path]
        name = f"{self.job.name}-trainer-0"
        pid = self.launcher.spawn(name, argv, env=self._base_env(), cwd=REPO_ROOT,
                                  log_path=os.path.join(self.run_dir, "logs", f"{name}.log"))
        self.procs[name] = Proc(name, "trainer", 0, pid, None, Resource(), time.time())
        self.events.emit("spawn", name=name, pid=pid, role="trainer")
        if self.kv is None:
            self.kv = self._connect_master()
        if self.desired is not None and self.master_argv is not None:
            self.kv.set("jobresource", json.dumps(self.desired.to_dict()))

    def _connect_master(self, timeout_s: float = 120.0):
        from easydl_amd.master.store import KV, make_tcp_store
        t_end = time.time() + timeout_s
        last = None
        while time.time() < t_end:
            try:
                st = make_tcp_store("127.0.0.1", self.master_port, False, timeout_s=10)
                return KV(st, f"edl/{self.job.name}")
            except Exception as e:  # master not listening yet
                last = e
                time.sleep(0.2)
        raise RuntimeError(f"job master did not come up on port {self.master_port}: {last}")

    def _base_env(self) -> dict:
        env = dict(os.environ)
        env.update(self.job.env)
        env["PYTHONPATH"] = REPO_ROOT + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
        env.update({"EDL_JOB": self.job.name, "EDL_MASTER_ADDR": "127.0.0.1",
                    "EDL_MASTER_PORT": str(self.master_port), "EDL_RUN_DIR": self.run_dir})
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if max(self.cfg.standby, getattr(self.job, "standby", 0)) > 0:
            # workers export their state buffers, a standby adopts a dead one's (utils/vram.py)
            env.setdefault("EDL_VRAM_HANDOFF", "1")
        if hw_queues_capped(self.cfg.gpus, max(self.cfg.standby, getattr(self.job, "standby", 0))):
            # too many processes hold a context on one GPU: every process's streams beyond this
            # many share hardware queues.  With HIP's default (4 per process) the ranks, standbys
            # and replacements oversubscribe the queues the scheduler maps at once; it then
            # time-slices whole processes, and the engine's cross-process barriers stall across
            # slices: world-3 steps of 33-460 ms median after a kill + rejoin, 5.8 ms with 2
            # queues (profiles/r04_shared_gpu_rejoin_slowdown.md)
            env["GPU_MAX_HW_QUEUES"] = os.environ.get("EDL_SHARED_GPU_HW_QUEUES", "2")
        for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_USE_AGENT_STORE"):
            env.pop(k, None)
        return env

    # ------------------------------------------------------------- reconcile
    def _role_procs(self, role: str) -> list[Proc]:
        return [p for p in self.procs.values() if p.role == role and p.state in ("running", "leaving")]

    def _completed(self, role: str) -> int:
        return sum(1 for p in self.procs.values() if p.role == role and p.state == "completed")

    def _role_env(self, role: str, index: int, res: Resource, generation: int) -> tuple[dict, int | None, list]:
        """Environment delta, GPU and CPU set of one role incarnation."""
        env = {}
        gpu = None
        if self._needs_gpu(role, res):
            if self._free_gpus:
                gpu = self._free_gpus.pop(0)
                env["EDL_GPU"] = str(gpu)
        env.update({"EDL_ROLE": ROLE_SHORT[role], "EDL_INDEX": str(index), "EDL_GENERATION": str(generation)})
        if self.desired is not None and "parameter_server" in self.desired.roles:
            env["EDL_NUM_PS"] = str(self.desired.replicas("parameter_server"))  # shard count for PS jobs
        if res.cu:
            env["EDL_CU_MASK"] = cu_mask_hex(res.cu)
        if res.hbm_gb:
            env["EDL_HBM_GB"] = str(res.hbm_gb)
        cpus = []
        if res.cpu:
            # the role's CPU share bounds its intra-op threads even without pinning: N
            # processes x all-core OpenMP pools oversubscribe the host (measured: a 3-worker
            # CPU job ran 4.8 s steps instead of 8 ms)
            n = max(1, int(res.cpu))
            env["OMP_NUM_THREADS"] = str(n)
            if self.cfg.cpus:
                used = set()
                for p in list(self.procs.values()) + list(self.standbys.values()):
                    used |= set(getattr(p, "cpus", []))
                cpus = [c for c in self.cfg.cpus if c not in used][:n]
        return env, gpu, cpus

    def _argv_for(self, role: str) -> list[str]:
        cmd = self.job.command_for(role)
        if not cmd:
            raise ValueError(f"no command for role {role}")
        argv = shlex.split(cmd)
        if argv[0] in ("python", "python3"):
            argv[0] = self.cfg.python
        return argv

    def _spawn_role(self, role: str, index: int, res: Resource, generation: int = 0) -> Proc:
        name = f"{self.job.name}-{ROLE_SHORT[role]}-{index}"
        delta, gpu, cpus = self._role_env(role, index, res, generation)
        argv = self._argv_for(role)
        taken = self._take_standby(role, name, argv, delta, gpu, cpus, res, index, generation)
        if taken is not None:
            return taken
        env = self._base_env()
        env.update(delta)
        if role in [r.strip() for r in env.get("EDL_ROCPROF_ROLES", "").split(",") if r.strip()]:
            # kernel-stats profile of this incarnation for the Brain's CU plan
            # (brain/collectors.py::rocprof_rank_profiles reads <run_dir>/rocprof/<name>/)
            out = os.path.join(self.run_dir, "rocprof", name)
            argv = ["rocprofv3", "--kernel-trace", "--stats", "--output-format", "csv", "-d", out, "-o", "k",
                    "--", *argv]
        pid = self.launcher.spawn(name, argv, env=env, cwd=REPO_ROOT,
                                  log_path=os.path.join(self.run_dir, "logs", f"{name}.log"), cpus=cpus)
        p = Proc(name, role, index, pid, gpu, res, time.time(), generation=generation)
        p.cpus = cpus
        self.procs[name] = p
        self.events.emit("spawn", name=name, pid=pid, role=role, gpu=gpu, gen=generation, resource=res.to_dict())
        self._announce_arrival(p)
        return p

    def _announce_arrival(self, p: Proc) -> None:
        """Tell the rendezvous that a worker is starting (RendezvousManager.arriving): the
        master then admits all joiners of one scale event in ONE re-formation, even when
        their start-up and pre-join warm-up finish at different times."""
        if p.role != "worker" or self.kv is None:
            return
        try:
            self.kv.set(f"rdzv/arrive_ts/{p.node_id}", str(time.time()))
            self.kv.append("rdzv/arriving", p.node_id + ",")
        except Exception as e:  # the store is best effort here: the join window still applies
            log.debug("arrival announcement for %s failed: %s", p.node_id, e)

    # ------------------------------------------------------------- hot standby
    def _maintain_standbys(self) -> None:
        from easydl_amd.operator.standby import module_of
        want = max(self.cfg.standby, getattr(self.job, "standby", 0))
        if want <= 0 or self.kv is None or self.done:
            return
        try:
            mod = module_of(self._argv_for("worker"))
        except ValueError:
            return
        if mod is None:
            return  # not a `python -m` entry: a standby could not run it in-process
        if time.time() - self._last_takeover < 20.0:
            return  # refill later: a starting spare would compete for CPUs with the replacement's restore
        while len(self.standbys) < want:
            name = f"{self.job.name}-standby-{self._standby_seq}"
            self._standby_seq += 1
            env = self._base_env()
            env.update({"EDL_STANDBY_NAME": name, "EDL_STANDBY_MODULE": mod, "EDL_ROLE": "standby"})
            argv = [self.cfg.python, "-m", "easydl_amd.operator.standby"]
            pid = self.launcher.spawn(name, argv, env=env, cwd=REPO_ROOT,
                                      log_path=os.path.join(self.run_dir, "logs", f"{name}.log"))
            self.standbys[name] = Proc(name, "standby", self._standby_seq - 1, pid, None, Resource(), time.time())
            self.events.emit("standby_spawn", name=name, pid=pid)

    def _publish_roster(self) -> None:
        """``standby/roster``: the parked standbys that are ready to take over.  Workers wait for
        their warm-up before the first step, and the fault drills for it before the kill
        (utils/vram.py standby_warm_on); a standby that took over leaves the roster at once."""
        if self.kv is None:
            return
        ready = []
        for sname in sorted(self.standbys):
            if sname in self._ready_seen:
                ready.append(sname)
                continue
            try:
                if self.kv.get(f"standby/ready/{sname}"):
                    self._ready_seen.add(sname)
                    ready.append(sname)
            except Exception:  # noqa: BLE001 - store unreachable: keep the last roster
                return
        roster = ",".join(ready)
        # spawned but not ready yet (still importing): a worker about to take its first step waits
        # for their warm-up too (standby_warm_on), instead of racing a standby that is coming
        pending = ",".join(n for n in sorted(self.standbys) if n not in ready)
        if (roster, pending) != (self._roster, getattr(self, "_pending", None)):
            try:
                self.kv.set("standby/pending", pending)
                self.kv.set("standby/roster", roster)
                self._roster, self._pending = roster, pending
            except Exception:  # noqa: BLE001
                pass

    def _standby_ready(self) -> bool:
        if self.kv is None:
            return False
        for sname in list(self.standbys):
            try:
                if self.kv.get(f"standby/ready/{sname}"):
                    return True
            except Exception:  # noqa: BLE001 - store unreachable: no standby to count on
                return False
        return False

    def _take_standby(self, role, name, argv, delta, gpu, cpus, res, index, generation) -> Proc | None:
        from easydl_amd.operator.standby import module_of
        if role != "worker" or not self.standbys or self.kv is None or module_of(argv) is None:
            return None
        for sname, sp in list(self.standbys.items()):
            try:
                ready = self.kv.get(f"standby/ready/{sname}")
            except Exception:
                ready = None
            if not ready:
                continue
            env = dict(self.job.env)
            env.update(delta)
            self.kv.set(f"standby/assign/{sname}", json.dumps({"env": env, "argv": argv}))
            if cpus:
                try:
                    os.sched_setaffinity(sp.pid, cpus)
                except OSError:
                    pass
            del self.standbys[sname]
            self._publish_roster()
            self._last_takeover = time.time()
            p = Proc(name, role, index, sp.pid, gpu, res, time.time(), generation=generation)
            p.cpus = cpus
            p.standby = sname
            self.procs[name] = p
            self.events.emit("spawn", name=name, pid=sp.pid, role=role, gpu=gpu, gen=generation,
                             resource=res.to_dict(), standby=sname)
            self._announce_arrival(p)
            return p
        return None

    def _needs_gpu(self, role: str, res: Resource) -> bool:
        if res.gpu is not None:
            return res.gpu > 0
        return role == "worker" and bool(self.cfg.gpus)

    def reconcile(self) -> None:
        jr = self.desired
        if jr is None:
            return
        # vertical scaling by replacement (reference :99-101): the old incarnation
        # leaves at its next step boundary; the new one starts with the merged
        # resource as soon as its GPU is free.
        for u in jr.resource_updation:
            key = (jr.version, u.name)
            if key in self.applied_updations:
                continue
            old = self.procs.get(u.name)
            if old is None or old.state != "running":
                continue
            self.applied_updations.add(key)
            self.overrides[u.name] = old.resource.merged(u.resource)
            self._begin_leave(old, replaced=True)
            del self.procs[old.name]
            self.history.append(old)
            self.events.emit("replace", name=u.name, resource=self.overrides[u.name].to_dict())
        for role, rr in jr.roles.items():
            running = [p for p in self._role_procs(role) if p.state == "running"]
            want = max(0, rr.replicas - self._completed(role))
            if len(running) < want:
                used = {p.index for p in self.procs.values() if p.role == role}
                idx = 0
                for _ in range(want - len(running)):
                    while idx in used:
                        idx += 1
                    name = f"{self.job.name}-{ROLE_SHORT[role]}-{idx}"
                    res = self.overrides.get(name, rr.resource)
                    if self._needs_gpu(role, res) and not self._free_gpus:
                        break  # wait for a GPU to be released
                    prev = [h for h in self.history if h.name == name]
                    gen = (max(h.generation for h in prev) + 1) if prev else 0
                    self._spawn_role(role, idx, res, gen)
                    used.add(idx)
            elif len(running) > want:
                for p in sorted(running, key=lambda p: -p.index)[:len(running) - want]:
                    self._begin_leave(p)

    def _begin_leave(self, p: Proc, replaced: bool = False) -> None:
        if p.state != "running":
            return
        p.state = "replaced" if replaced else "leaving"
        p.leave_ts = time.time()
        if self.kv is not None and p.role != "trainer":
            self.kv.set(f"rdzv/leave/{p.node_id}", "1")
        self.events.emit("leave", name=p.name, replaced=replaced)

    def _release_gpu(self, p: Proc) -> None:
        # cfg.gpus may list an ordinal several times (slots of one shared GPU); a process
        # gives its slot back once (p.gpu is cleared)
        if p.gpu is not None:
            self._free_gpus.append(p.gpu)
            self._free_gpus.sort()
            p.gpu = None

    def _enforce_grace(self):
        now = time.time()
        for p in list(self.procs.values()) + self.history:
            if p.state in ("leaving", "replaced") and now - getattr(p, "leave_ts", now) > self.cfg.leave_grace_s:
                try:
                    self.launcher.kill(p.pid, signal.SIGKILL)
                except OSError:
                    pass

    # ------------------------------------------------------------- events
    def handle_exit(self, ex) -> None:
        sb = next((q for q in self.standbys.values() if q.pid == ex.pid), None)
        if sb is not None:
            del self.standbys[sb.name]
            self._publish_roster()
            self.events.emit("standby_exit", name=sb.name, code=ex.exit_code, signal=ex.signal)
            return
        p = next((q for q in list(self.procs.values()) + self.history if q.pid == ex.pid), None)
        if p is None:
            return
        if getattr(p, "_early_replaced", False):   # already replaced when its address space went away
            self.events.emit("exit", name=p.name, pid=p.pid, code=ex.exit_code, signal=ex.signal, role=p.role,
                             early=True)
            return
        p.exit_code = ex.exit_code if not ex.signal else -ex.signal
        self.events.emit("exit", name=p.name, pid=p.pid, code=ex.exit_code, signal=ex.signal, role=p.role)
        if self.kv is not None:
            self.kv.delete(f"metrics/{p.node_id}")   # the plan loop must not re-plan a process that is gone
        if p.role == "trainer":
            p.state = "exited"
            if not self.done:
                self.failed = ex.exit_code != 0 or ex.signal != 0
            return
        if self.kv is not None:
            try:
                self.kv.set(f"ev/exit/{p.node_id}", json.dumps({"code": ex.exit_code, "signal": ex.signal,
                                                                 "ts": ex.ts}))
            except Exception:
                pass
        self._release_gpu(p)
        if p.state in ("leaving", "replaced"):
            p.state = "exited"
            if self.procs.get(p.name) is p:
                del self.procs[p.name]
                self.history.append(p)
            return
        if ex.exit_code == 0 and not ex.signal:
            p.state = "completed"
            return
        p.state = "exited"
        self.restarts += 1
        if self.procs.get(p.name) is p:
            del self.procs[p.name]
            self.history.append(p)
        if not self.cfg.replace_failed or self.restarts > self.cfg.max_restarts:
            log.error("not replacing %s (restarts %d)", p.name, self.restarts)

    def _poll_jobresource(self) -> None:
        if self.kv is None:
            return
        try:
            raw = self.kv.get("jobresource")
        except Exception:
            return
        if raw is None:
            return
        doc = raw if isinstance(raw, dict) else json.loads(raw)
        from easydl_amd.api.schema import validate
        errs = validate(doc, "JobResource")
        if errs:
            if doc.get("spec", {}).get("version") != getattr(self, "_rejected_version", None):
                self._rejected_version = doc.get("spec", {}).get("version")
                log.error("JobResource rejected by schema: %s", errs)
                self.events.emit("jobresource_rejected", errors=errs[:8])
            return
        jr = JobResource.from_dict(doc)
        if jr.selector != self.job.name:
            log.error("JobResource selector %s does not match job %s: ignored", jr.selector, self.job.name)
            return
        if self.desired is None or jr.version != self.applied_version or jr.to_dict() != self.desired.to_dict():
            self.desired = jr
            self.applied_version = jr.version
            self.events.emit("jobresource_applied", version=jr.version,
                             replicas={r: v.replicas for r, v in jr.roles.items()})

    def job_complete(self) -> bool:
        jr = self.desired
        if jr is None:
            return False
        workers = [p for p in self.procs.values() if p.role == "worker"]
        return jr.replicas("worker") > 0 and bool(workers) and all(p.state == "completed" for p in workers)

    def _early_exits(self) -> None:
        """Report deaths as soon as the kernel starts tearing a worker down."""
        if not hasattr(self.launcher, "exiting") or self.kv is None:
            return
        for pid in self.launcher.exiting():
            p = next((q for q in self.procs.values() if q.pid == pid), None)
            if p is None or p.role == "trainer" or getattr(p, "_early_reported", False):
                continue
            p._early_reported = True
            if p.state == "running":
                try:
                    self.kv.set(f"ev/exit/{p.node_id}", json.dumps({"exiting": True, "ts": time.time()}))
                    self.events.emit("exiting", name=p.name, pid=pid)
                except Exception:
                    pass

    def _early_replace(self) -> None:
        """Replace a dying worker once its address space is gone, before the kernel has torn
        it down and reaped it.  The GPU's queues of a process are destroyed at the start of
        its address-space teardown (the amdkfd MMU-notifier release), but tearing down the
        page tables of a large mapped snapshot segment takes ~19 ms per GB after that
        (scripts/exit_cost_probe.cpp); the replacement does not wait for it.  A replacement
        that adopted the dead worker's HBM re-verifies its restored state once the dead
        process is reaped, before its first optimizer step (ckpt/manager.py fence).  Only when
        a parked standby is ready to take over: it builds on the dead worker's HBM (utils/vram.py),
        while a freshly started process would allocate it and run out of memory until the dead
        one's HBM is released.  EDL_EARLY_HANDOVER=0: wait for the reap as before."""
        if os.environ.get("EDL_EARLY_HANDOVER", "1") == "0":
            return
        now = time.time()
        for p in list(self.procs.values()):
            if p.role != "worker" or p.state != "running" or not getattr(p, "_early_reported", False):
                continue
            if not mm_released(p.pid):
                continue
            if not exit_status(p.pid):   # a normal exit(0) (or unknown): its reap decides, as before
                continue
            if not self._standby_ready():
                continue
            t = getattr(p, "_mm_gone_ts", None)
            if t is None:
                p._mm_gone_ts = now
                continue
            if now - t < 0.1:   # grace for the driver's queue teardown
                continue
            p._early_replaced = True
            st = exit_status(p.pid) or 0
            p.exit_code = -(st & 0x7F) if st & 0x7F else (st >> 8) & 0xFF
            self.events.emit("exit_early", name=p.name, pid=p.pid, role=p.role, mm_gone_s=round(now - t, 3))
            self._release_gpu(p)
            p.state = "exited"
            self.restarts += 1
            if self.procs.get(p.name) is p:
                del self.procs[p.name]
                self.history.append(p)

    def tick(self, timeout_s: float = 0.05) -> None:
        self._early_exits()
        self._early_replace()
        for ex in self.launcher.poll(timeout_s):
            self.handle_exit(ex)
        self._poll_jobresource()
        self.reconcile()
        self._maintain_standbys()
        self._publish_roster()
        self._enforce_grace()
        if self.job_complete() and not self.done:
            self.done = True
            self.events.emit("job_complete")

    def run(self, timeout_s: float | None = None) -> int:
        self.start()
        t_end = None if timeout_s is None else time.time() + timeout_s
        try:
            while not self.done and not self.failed:
                self.tick()
                if t_end is not None and time.time() > t_end:
                    log.error("operator timeout")
                    return 2
        finally:
            self.shutdown()
        return 0 if self.done else 1

    def shutdown(self) -> None:
        if self.kv is not None:
            try:
                self.kv.set("job/done", "1")      # PS / evaluator roles exit on their own
                t_end = time.time() + 5
                while time.time() < t_end and any(p.state == "running" and p.role in ("parameter_server",
                                                                                        "evaluator")
                                                  for p in self.procs.values()):
                    for ex in self.launcher.poll(0.1):
                        self.handle_exit(ex)
                self.kv.set("master/shutdown", "1")
            except Exception:
                pass
        for p in list(self.standbys.values()):
            try:
                self.launcher.terminate(p.pid, grace_s=2.0)
            except Exception:
                pass
        for p in list(self.procs.values()):
            if p.state in ("running", "leaving", "replaced"):
                try:
                    self.launcher.terminate(p.pid, grace_s=5.0)
                except Exception:
                    pass
        if hasattr(self.launcher, "close"):
            self.launcher.close()
