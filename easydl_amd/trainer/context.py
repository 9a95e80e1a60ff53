"""Process context: the ``EDL_*`` environment contract set by the local
ElasticOperator (or derived from ``torchrun``'s variables).

==================  =====================================================
EDL_JOB             job name (store key prefix, process names)
EDL_ROLE            trainer | worker | ps | evaluator
EDL_INDEX           role index (``<job>-<role>-<index>``, reference naming
                    ``docs/design/elastic-training-operator.md:87``)
EDL_MASTER_ADDR     host of the job master's TCPStore
EDL_MASTER_PORT     its port
EDL_RUN_DIR         directory for events / metrics / checkpoints
EDL_GPU             GPU ordinal this process drives (HIP_VISIBLE_DEVICES
                    may also be set by the operator)
EDL_CU_MASK         optional CU mask (hex) from the Brain plan
EDL_HBM_GB          optional HBM cap from the Brain plan
EDL_FAULT           fault-injection spec (easydl_amd.utils.fault)
==================  =====================================================
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field


@dataclass
class TrainerContext:
    job: str = "job"
    role: str = "worker"
    index: int = 0
    master_addr: str | None = None
    master_port: int | None = None
    run_dir: str = "runs/job"
    gpu: int | None = None
    embedded_master: bool = False    # rank 0 of a torchrun job hosts the rendezvous manager
    static_world: int | None = None  # torchrun WORLD_SIZE
    cu_mask: str | None = None
    hbm_gb: float | None = None
    env: dict = field(default_factory=dict)

    @property
    def node_id(self) -> str:
        return f"{self.job}-{self.role}-{self.index}:{os.getpid()}"

    @property
    def standalone(self) -> bool:
        return self.master_addr is None

    @classmethod
    def from_env(cls, env=None) -> "TrainerContext":
        e = dict(os.environ if env is None else env)
        job = e.get("EDL_JOB", "job")
        ctx = cls(job=job, role=e.get("EDL_ROLE", "worker"), index=int(e.get("EDL_INDEX", e.get("RANK", 0))),
                  run_dir=e.get("EDL_RUN_DIR", os.path.join("runs", job)), env=e)
        if "EDL_MASTER_ADDR" in e:
            ctx.master_addr = e["EDL_MASTER_ADDR"]
            ctx.master_port = int(e.get("EDL_MASTER_PORT", 29400))
        elif "WORLD_SIZE" in e and int(e.get("WORLD_SIZE", 1)) > 1:
            # launched by torchrun: reuse its store, rank 0 embeds the master
            ctx.master_addr = e.get("MASTER_ADDR", "127.0.0.1")
            ctx.master_port = int(e.get("MASTER_PORT", 29500))
            ctx.embedded_master = True
            ctx.static_world = int(e["WORLD_SIZE"])
        if "EDL_GPU" in e:
            ctx.gpu = int(e["EDL_GPU"])
        elif "LOCAL_RANK" in e:
            ctx.gpu = int(e["LOCAL_RANK"])
        ctx.cu_mask = e.get("EDL_CU_MASK")
        ctx.hbm_gb = float(e["EDL_HBM_GB"]) if "EDL_HBM_GB" in e else None
        return ctx
