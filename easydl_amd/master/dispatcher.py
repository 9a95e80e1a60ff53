"""Elastic data dispatch for parameter-server jobs.

The dataset index space is cut into shards of ``shard_size`` samples.  Workers
claim shards from the job master's store (an atomic cursor) and hold a lease
``data/lease/<shard> = <node>`` while they work on it; completing a shard
removes the lease.  When a worker dies the master requeues every shard it
still leased (``data/requeue`` log + per-entry claim keys), so no sample is
lost and none is processed twice inside an epoch — the "resume the training"
half of failure recovery (reference README.md:27) for PS mode.  All-reduce
jobs use the step-indexed :class:`easydl_amd.trainer.data.ElasticBatchPlan`
instead.
"""
from __future__ import annotations



class ShardDispatcher:
    def __init__(self, kv, num_samples: int, shard_size: int, epochs: int = 1):
        self.kv = kv
        self.n = num_samples
        self.shard_size = shard_size
        self.num_shards = (num_samples + shard_size - 1) // shard_size
        self.epochs = epochs

    @property
    def total(self) -> int:
        return self.num_shards * self.epochs

    def shard_range(self, shard: int) -> tuple[int, int]:
        s = shard % self.num_shards
        return s * self.shard_size, min(self.n, (s + 1) * self.shard_size)

    # -- worker side -----------------------------------------------------------
    def claim(self, node: str) -> int | None:
        """Next shard for ``node`` (requeued ones first); None when the job's data is exhausted."""
        raw = self.kv.get_str("data/requeue", "") or ""
        for tok in filter(None, raw.split(",")):
            ck = f"data/requeue_claim/{tok}"
            if self.kv.exists(ck):  # claimed already (possibly by us earlier)
                continue
            if self.kv.compare_set(ck, "", node) == node:
                shard = int(tok.split(":")[0])
                self.kv.set(f"data/lease/{shard}", node)
                return shard
        shard = self.kv.add("data/cursor", 1) - 1
        if shard >= self.total:
            return None
        self.kv.set(f"data/lease/{shard}", node)
        return shard

    def complete(self, shard: int) -> None:
        self.kv.delete(f"data/lease/{shard}")
        self.kv.add("data/done", 1)

    def done(self) -> int:
        return self.kv.counter("data/done")

    # -- master side -------------------------------------------------------------
    def requeue_dead(self, dead_nodes: set[str]) -> list[int]:
        out = []
        hi = min(self.total, self.kv.counter("data/cursor"))
        for shard in range(hi):
            owner = self.kv.get_str(f"data/lease/{shard}")
            if owner is not None and owner in dead_nodes:
                n = self.kv.add(f"data/requeue_n/{shard}", 1)
                self.kv.append("data/requeue", f"{shard}:{n},")
                self.kv.delete(f"data/lease/{shard}")
                out.append(shard)
        return out
