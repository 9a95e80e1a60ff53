"""Job specifications: ElasticJob, JobResource, Resource, ResourcePlan.

Schema parity with the reference CRDs (docs/design/elastic-training-operator.md):

* ``ElasticJob`` (:31-45) — job name, trainer ``image``, ``command`` and per-role
  images for ``parameter_server`` / ``worker`` / ``evaluator``; **no resources
  or replicas** (:27-29: the user need not configure any).
* ``JobResource`` (:57-95) — ``selector.name`` binds it to a job (:63-64);
  per-role ``replicas`` + ``resource{cpu, memory, disk, gpu}``; and
  ``resource_updation: [{name, resource}]`` replaces the named process with a
  new one carrying the new resource (:86-101).

Both accept the reference ``apiVersion: elastic.easydl.org/v1alpha1`` and our
``edl.mi355x/v1``.  Reference quirks are resolved explicitly (SURVEY.md
Appendix B): ``// comment`` suffixes inside values are stripped with a warning;
memory/disk units are MiB.  MI355X extensions on Resource: ``cu`` (CUs of the
256 to mask the role's streams to), ``hbm_gb`` (allocator cap), and plan-level
``bucket_mb`` / ``ckpt_interval``.  On this single-node re-cast an "image" is
an execution environment hint (python interpreter / venv); ``command`` is what
runs (``python -m easydl_amd.examples.mnist`` etc.).
"""
from __future__ import annotations

import copy
import json
import logging
import os
from dataclasses import asdict, dataclass, field

import yaml

log = logging.getLogger(__name__)

API_VERSIONS = ("elastic.easydl.org/v1alpha1", "edl.mi355x/v1")
ROLES = ("parameter_server", "worker", "evaluator")
ROLE_SHORT = {"parameter_server": "ps", "worker": "worker", "evaluator": "evaluator", "trainer": "trainer"}


class SpecError(ValueError):
    pass


def _clean(v):
    """Strip the reference's non-YAML ``// comment`` suffixes (docs/...md:64)."""
    if isinstance(v, str) and "//" in v:
        head = v.split("//", 1)[0].strip()
        log.warning("stripping '//' comment from spec value %r", v)
        return head
    return v


def _num(v, kind=float):
    v = _clean(v)
    if v is None or v == "":
        return None
    return kind(v)


@dataclass
class Resource:
    cpu: float | None = None
    memory: float | None = None   # MiB
    disk: float | None = None     # MiB
    gpu: int | None = None
    cu: int | None = None         # MI355X: compute units (of 256) for the role's streams
    hbm_gb: float | None = None   # MI355X: HBM allocator cap per process

    @classmethod
    def from_dict(cls, d: dict | None) -> "Resource":
        d = d or {}
        unknown = set(d) - {"cpu", "memory", "disk", "gpu", "cu", "hbm_gb"}
        if unknown:
            raise SpecError(f"unknown resource fields {sorted(unknown)}")
        r = cls(cpu=_num(d.get("cpu")), memory=_num(d.get("memory")), disk=_num(d.get("disk")),
                gpu=_num(d.get("gpu"), int), cu=_num(d.get("cu"), int), hbm_gb=_num(d.get("hbm_gb")))
        r.validate()
        return r

    def validate(self):
        for k in ("cpu", "memory", "disk", "gpu", "cu", "hbm_gb"):
            v = getattr(self, k)
            if v is not None and v < 0:
                raise SpecError(f"resource.{k} must be >= 0")
        if self.cu is not None and self.cu > 256:
            raise SpecError("resource.cu cannot exceed 256 CUs of an MI355X")
        if self.hbm_gb is not None and self.hbm_gb > 288:
            raise SpecError("resource.hbm_gb cannot exceed 288 GB")

    def merged(self, other: "Resource") -> "Resource":
        """Fields set in ``other`` override ours (partial updates, docs/...md:88-94)."""
        out = copy.copy(self)
        for k, v in asdict(other).items():
            if v is not None:
                setattr(out, k, v)
        return out

    def to_dict(self) -> dict:
        return {k: v for k, v in asdict(self).items() if v is not None}


@dataclass
class RoleSpec:
    image: str = ""
    command: str | None = None


@dataclass
class ElasticJob:
    name: str
    command: str = ""
    image: str = ""
    roles: dict[str, RoleSpec] = field(default_factory=dict)
    api_version: str = API_VERSIONS[1]
    # easydl_amd extensions (optional)
    mode: str = "allreduce"          # allreduce | ps
    env: dict = field(default_factory=dict)
    min_workers: int = 1
    max_workers: int = 8
    features: dict = field(default_factory=dict)   # hints for the Brain (model name, seq, batch...)
    standby: int = 0    # warm spare worker processes kept parked by the operator (hot standby)

    @classmethod
    def from_dict(cls, d: dict) -> "ElasticJob":
        if d.get("kind", "ElasticJob") != "ElasticJob":
            raise SpecError(f"expected kind ElasticJob, got {d.get('kind')}")
        av = d.get("apiVersion", API_VERSIONS[1])
        if av not in API_VERSIONS:
            raise SpecError(f"unsupported apiVersion {av}")
        name = _clean((d.get("metadata") or {}).get("name"))
        if not name:
            raise SpecError("metadata.name is required")
        spec = d.get("spec") or {}
        roles = {}
        for r in ROLES:
            if r in spec and spec[r] is not None:
                rs = spec[r] or {}
                roles[r] = RoleSpec(image=_clean(rs.get("image") or ""), command=_clean(rs.get("command")))
        if "resources" in spec or any(isinstance(spec.get(r), dict) and "replicas" in spec[r] for r in ROLES):
            raise SpecError("ElasticJob carries no resources/replicas: put them in a JobResource")
        return cls(name=name, command=_clean(spec.get("command") or ""), image=_clean(spec.get("image") or ""),
                   roles=roles, api_version=av, mode=spec.get("mode", "ps" if "parameter_server" in roles else
                                                              "allreduce"),
                   env=dict(spec.get("env") or {}), min_workers=int(spec.get("min_workers", 1)),
                   max_workers=int(spec.get("max_workers", 8)), features=dict(spec.get("features") or {}),
                   standby=int(spec.get("standby", 0)))

    def to_dict(self) -> dict:
        spec = {"command": self.command, "image": self.image}
        for r, rs in self.roles.items():
            spec[r] = {"image": rs.image} | ({"command": rs.command} if rs.command else {})
        spec.update(mode=self.mode, env=self.env, min_workers=self.min_workers, max_workers=self.max_workers,
                    features=self.features, standby=self.standby)
        return {"apiVersion": self.api_version, "kind": "ElasticJob", "metadata": {"name": self.name}, "spec": spec}

    def command_for(self, role: str) -> str:
        rs = self.roles.get(role)
        return (rs.command if rs and rs.command else None) or self.command


@dataclass
class RoleResource:
    replicas: int = 0
    resource: Resource = field(default_factory=Resource)


@dataclass
class ResourceUpdation:
    name: str
    resource: Resource


@dataclass
class JobResource:
    name: str
    selector: str
    roles: dict[str, RoleResource] = field(default_factory=dict)
    resource_updation: list[ResourceUpdation] = field(default_factory=list)
    api_version: str = API_VERSIONS[1]
    # plan-level MI355X knobs
    bucket_mb: float | None = None
    ckpt_interval: int | None = None
    allreduce: dict | None = None      # all-reduce routing policy (parallel/comm_policy.py)
    version: int = 0

    @classmethod
    def from_dict(cls, d: dict) -> "JobResource":
        if d.get("kind", "JobResource") != "JobResource":
            raise SpecError(f"expected kind JobResource, got {d.get('kind')}")
        av = d.get("apiVersion", API_VERSIONS[1])
        if av not in API_VERSIONS:
            raise SpecError(f"unsupported apiVersion {av}")
        spec = d.get("spec") or {}
        sel = _clean((spec.get("selector") or {}).get("name"))
        if not sel:
            raise SpecError("spec.selector.name (the ElasticJob name) is required")
        roles = {}
        for r in ROLES:
            if r in spec and spec[r] is not None:
                rr = spec[r]
                reps = _num(rr.get("replicas"), int) or 0
                if reps < 0:
                    raise SpecError(f"{r}.replicas must be >= 0")
                roles[r] = RoleResource(replicas=reps, resource=Resource.from_dict(rr.get("resource")))
        upd = []
        for u in spec.get("resource_updation") or []:
            upd.append(ResourceUpdation(name=_clean(u["name"]), resource=Resource.from_dict(u.get("resource"))))
        return cls(name=_clean((d.get("metadata") or {}).get("name") or f"{sel}-resource"), selector=sel,
                   roles=roles, resource_updation=upd, api_version=av, bucket_mb=_num(spec.get("bucket_mb")),
                   ckpt_interval=_num(spec.get("ckpt_interval"), int), allreduce=spec.get("allreduce") or None,
                   version=int(spec.get("version", 0)))

    def to_dict(self) -> dict:
        spec = {"selector": {"name": self.selector}}
        for r, rr in self.roles.items():
            spec[r] = {"replicas": rr.replicas, "resource": rr.resource.to_dict()}
        if self.resource_updation:
            spec["resource_updation"] = [{"name": u.name, "resource": u.resource.to_dict()}
                                         for u in self.resource_updation]
        if self.bucket_mb is not None:
            spec["bucket_mb"] = self.bucket_mb
        if self.ckpt_interval is not None:
            spec["ckpt_interval"] = self.ckpt_interval
        if self.allreduce:
            spec["allreduce"] = self.allreduce
        spec["version"] = self.version
        return {"apiVersion": self.api_version, "kind": "JobResource", "metadata": {"name": self.name},
                "spec": spec}

    def replicas(self, role: str) -> int:
        rr = self.roles.get(role)
        return rr.replicas if rr else 0


@dataclass
class ResourcePlan:
    """Brain output (README.md:13 "resources plans")."""
    roles: dict[str, RoleResource] = field(default_factory=dict)
    per_rank: dict[str, dict] = field(default_factory=dict)   # process name -> {cu, hbm_gb, cpus}
    bucket_mb: float | None = None
    ckpt_interval: int | None = None
    allreduce: dict | None = None      # {"dp"|"tp": {"world", "epochs", "policy"}} from the probe history
    reason: str = ""

    def to_job_resource(self, job: str, version: int = 0) -> JobResource:
        return JobResource(name=f"{job}-resource", selector=job, roles=copy.deepcopy(self.roles),
                           bucket_mb=self.bucket_mb, ckpt_interval=self.ckpt_interval,
                           allreduce=copy.deepcopy(self.allreduce), version=version)

    def to_dict(self) -> dict:
        return {"roles": {r: {"replicas": rr.replicas, "resource": rr.resource.to_dict()}
                          for r, rr in self.roles.items()},
                "per_rank": self.per_rank, "bucket_mb": self.bucket_mb, "ckpt_interval": self.ckpt_interval,
                "allreduce": self.allreduce, "reason": self.reason}

    @classmethod
    def from_dict(cls, d: dict) -> "ResourcePlan":
        roles = {r: RoleResource(int(v.get("replicas", 0)), Resource.from_dict(v.get("resource")))
                 for r, v in (d.get("roles") or {}).items()}
        return cls(roles=roles, per_rank=dict(d.get("per_rank") or {}), bucket_mb=d.get("bucket_mb"),
                   ckpt_interval=d.get("ckpt_interval"), allreduce=d.get("allreduce"), reason=d.get("reason", ""))


def load_yaml_docs(path_or_text: str) -> list[dict]:
    text = open(path_or_text).read() if os.path.exists(path_or_text) else path_or_text
    return [d for d in yaml.safe_load_all(text) if d]


def load_specs(path_or_text: str) -> tuple[ElasticJob | None, JobResource | None]:
    job = jr = None
    for d in load_yaml_docs(path_or_text):
        kind = d.get("kind")
        if kind == "ElasticJob":
            job = ElasticJob.from_dict(d)
        elif kind == "JobResource":
            jr = JobResource.from_dict(d)
        else:
            raise SpecError(f"unknown kind {kind}")
    if job is not None and jr is not None and jr.selector != job.name:
        raise SpecError(f"JobResource selector {jr.selector!r} does not match job {job.name!r}")
    return job, jr


def dumps(obj) -> str:
    return json.dumps(obj.to_dict())
