"""The trainer master's plan loop (reference docs/design/elastic-training-operator.md:105-112):

1. extract job features, query the Brain for *startup resources*, generate and
   apply a JobResource (written to the store key ``jobresource``, which the
   local ElasticOperator watches) — unless the user supplied one;
2. periodically collect per-rank metrics (``metrics/<node>``), ask the Brain
   for a new plan and update the JobResource (scale, replace stragglers via
   ``resource_updation``) and the runtime knobs (bucket size, checkpoint
   interval, all-reduce routing policy) that the trainers pick up at step
   boundaries.  The epochs' all-reduce probe tables (``comm/probe/dp`` and
   ``comm/probe/tp``, written by rank 0 of each group) go to the Brain with the metrics.

Runtime knobs travel as ONE versioned document, ``plan/runtime/<v>``, written
before the counter ``plan/version`` moves to ``v``: every rank switches to the
version its step commit agreed on and reads exactly that document, so a plan
applied between two ranks' reads can never give them different bucket layouts.
"""
from __future__ import annotations

import json
import logging
import time

from easydl_amd.api.spec import ElasticJob, JobResource, ResourcePlan, ResourceUpdation, Resource
from easydl_amd.brain.service import BrainClient

log = logging.getLogger("edl.master.plan")


class PlanLoop:
    def __init__(self, job: ElasticJob, brain: BrainClient | None = None, period_s: float = 30.0,
                 user_wait_s: float = 0.5):
        self.job = job
        self.brain = brain or BrainClient()
        self.period_s = period_s
        self.user_wait_s = user_wait_s
        self.plan: ResourcePlan | None = None
        self.version = 0
        self._t_start = time.time()
        self._last = 0.0
        self.started = False
        self._features = None
        # resource_updation issued per process name -> (node id it was issued for, time): not
        # issued again until a new incarnation of that name reports its metrics
        self._updating: dict[str, tuple[str, float]] = {}

    def features(self) -> dict:
        """Extracted job features (meta-device model analysis) + the user's hints."""
        if self._features is None:
            from easydl_amd.master.features import extract
            self._features = extract(self.job)
        return dict(self._features)

    def _apply(self, master, jr: JobResource):
        self.version += 1
        jr.version = self.version
        master.kv.set("jobresource", json.dumps(jr.to_dict()))
        # only the master moves plan/version: the next value is counter + 1
        nxt = master.kv.counter("plan/version") + 1
        master.kv.set(f"plan/runtime/{nxt}", json.dumps({"bucket_mb": jr.bucket_mb, "ckpt_interval": jr.ckpt_interval,
                                                          "allreduce": jr.allreduce}))
        master.kv.add("plan/version", 1)
        wr = jr.roles.get("worker")
        if wr is not None and self.job.mode == "allreduce":
            master.rdzv.target_nodes = wr.replicas
        master.events.emit("plan_applied", version=self.version, replicas={r: v.replicas for r, v in
                                                                             jr.roles.items()})

    def _adopt_external(self, master) -> None:
        """A JobResource written by someone else (``edl scale`` / ``edl apply`` / a user
        tool) supersedes the plan: follow its worker target so the rendezvous grows or
        shrinks the world to it (the operator already reconciles the processes)."""
        raw = master.kv.get("jobresource")
        if raw is None:
            return
        doc = raw if isinstance(raw, dict) else json.loads(raw)
        ver = int((doc.get("spec") or {}).get("version", 0))
        if ver == self.version:
            return
        jr = JobResource.from_dict(doc)
        self.version = ver
        if self.plan is not None:
            self.plan.roles = jr.roles
        wr = jr.roles.get("worker")
        if wr is not None and self.job.mode == "allreduce":
            master.rdzv.target_nodes = wr.replicas
        master.events.emit("jobresource_adopted", version=ver, replicas={r: v.replicas for r, v in jr.roles.items()})

    def maybe_replan(self, master) -> None:
        now = time.time()
        if not self.started:
            if master.kv.exists("jobresource"):
                raw = master.kv.get("jobresource")
                jr = JobResource.from_dict(raw if isinstance(raw, dict) else json.loads(raw))
                self.version = jr.version
                self.started = True
                self.plan = ResourcePlan(roles=jr.roles, bucket_mb=jr.bucket_mb, ckpt_interval=jr.ckpt_interval,
                                         allreduce=jr.allreduce, reason="user JobResource")
                wr = jr.roles.get("worker")
                if wr is not None and self.job.mode == "allreduce":
                    master.rdzv.target_nodes = wr.replicas
                return
            if now - self._t_start < self.user_wait_s:
                return
            self.plan = self.brain.startup_plan(self.features())
            master.events.emit("startup_plan", plan=self.plan.to_dict())
            self._apply(master, self.plan.to_job_resource(self.job.name))
            self.started = True
            self._last = now
            return
        self._adopt_external(master)
        if self.period_s <= 0 or now - self._last < self.period_s:
            return
        self._last = now
        # rendezvous members (workers) and the roles that registered their own metrics
        # (parameter servers, evaluators: utils/metrics.py publish_role_metrics); a role's record
        # older than a few periods belongs to a process that is gone
        extra = [n for n in (master.kv.get_str("metrics/extra_nodes") or "").split(",") if n]
        members = list(dict.fromkeys(master.rdzv.members() + extra))
        wall = time.time()
        fresh = wall - max(60.0, 3 * self.period_s)
        # (a record without a timestamp cannot be judged stale: kept)
        metrics = {n: m for n in members if (m := master.kv.get(f"metrics/{n}")) and m.get("ts", wall) >= fresh}
        if not metrics:
            return
        # rocprofv3 kernel profiles the roles left under <run_dir>/rocprof/<process>/ (Brain CU signal)
        from easydl_amd.brain.collectors import rocprof_rank_profiles
        profs = rocprof_rank_profiles(getattr(master, "run_dir", "") or "")
        for n in list(metrics):
            prof = profs.get(n.split(":")[0])
            if prof is not None:
                metrics[n] = dict(metrics[n], rocprof=prof)
        comm = {g: d for g in ("dp", "tp") if isinstance(d := master.kv.get(f"comm/probe/{g}"), dict)}
        newp = self.brain.next_plan(self.features(), self.plan, metrics, comm or None)
        if newp is None:
            return
        master.events.emit("replan", reason=newp.reason)
        jr = newp.to_job_resource(self.job.name)
        for node, d in newp.per_rank.items():
            name = node.split(":")[0]
            now = metrics.get(node) or {}
            pend = self._updating.get(name)
            if pend is not None and (pend[0] == node or time.time() - pend[1] < 5.0) \
                    and time.time() - pend[1] < 120.0:
                continue     # its replacement has not reported yet
            if d.get("evict"):
                jr.resource_updation.append(ResourceUpdation(name=name, resource=Resource()))
                continue
            res = Resource()
            if d.get("cu") and int(d["cu"]) != now.get("cu"):
                # CU plan from the rank's kernel mix (live, utils/kmix.py, or a rocprofv3 profile):
                # re-create it with CU-masked streams
                res.cu = int(d["cu"])
            if d.get("cpu") and int(d["cpu"]) != now.get("cpu"):
                res.cpu = float(d["cpu"])     # a CPU-bound parameter server gets more cores
            if d.get("hbm_gb") and float(d["hbm_gb"]) != now.get("hbm_cap_gb"):
                res.hbm_gb = float(d["hbm_gb"])   # HBM cap from the rank's measured allocator peak
            if res.cu or res.cpu or res.hbm_gb:
                jr.resource_updation.append(ResourceUpdation(name=name, resource=res))
        for u in jr.resource_updation:
            node = next((n for n in newp.per_rank if n.split(":")[0] == u.name), u.name)
            self._updating[u.name] = (node, time.time())
        for d in newp.per_rank.values():
            d.pop("evict", None)
        self.plan = newp
        self._apply(master, jr)
