"""Per-step training metrics (SURVEY.md §5.5, R12 "monitor the performance of a
training job"): rolling step-time window, throughput, memory; published to the
job master's store (``metrics/<node>``) where the Brain's periodic re-plan reads
them, appended to ``<run_dir>/metrics-<proc>.jsonl``, and rendered by the
master as Prometheus text (``render_prometheus``)."""
from __future__ import annotations

import json
import os
import statistics
import time
from collections import deque


class MetricsReporter:
    def __init__(self, kv=None, node: str = "", path: str | None = None, every: int = 10, window: int = 20):
        self.kv, self.node, self.path, self.every = kv, node, path, every
        self.times = deque(maxlen=window)
        self.n = 0
        self.last = {}
        if path:
            os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)

    def record(self, step: int, dt: float, samples: int = 0, tokens: int = 0, world: int = 1, loss=None,
               mem_gb: float | None = None, extra=None) -> dict | None:
        """``extra``: a dict, or a callable returning one, merged into the published record
        (evaluated only when a record is published, every ``every`` steps)."""
        self.times.append(dt)
        self.n += 1
        if self.n % self.every:
            return None
        st = statistics.median(self.times)
        m = {"step": step, "step_time": st, "window": len(self.times), "world": world, "ts": time.time(),
             "samples_per_s": samples / st if st else 0.0, "tokens_per_s": tokens / st if st else 0.0}
        if loss is not None:
            m["loss"] = float(loss)
        if mem_gb is not None:
            m["mem_gb"] = mem_gb
        if extra is not None:
            m.update({k: v for k, v in (extra() if callable(extra) else extra).items() if v is not None})
        self.last = m
        if self.kv is not None:
            try:
                self.kv.set(f"metrics/{self.node}", json.dumps(m))
            except Exception:
                pass
        if self.path:
            with open(self.path, "a") as f:
                f.write(json.dumps(m) + "\n")
        return m


def render_prometheus(metrics: dict[str, dict], job: str) -> str:
    lines = []
    for key in ("step_time", "tokens_per_s", "samples_per_s", "loss", "mem_gb", "step", "world"):
        lines.append(f"# TYPE edl_{key} gauge")
        for node, m in metrics.items():
            if key in m:
                lines.append(f'edl_{key}{{job="{job}",node="{node}"}} {m[key]}')
    return "\n".join(lines) + "\n"


def cu_count(mask_hex: str | None) -> int | None:
    """CUs enabled by an ``EDL_CU_MASK`` hex string (None: no mask, every CU)."""
    if not mask_hex:
        return None
    try:
        return bin(int(str(mask_hex), 16)).count("1")
    except ValueError:
        return None


def publish_role_metrics(kv, node: str, m: dict) -> None:
    """Metrics of a role that is not a rendezvous member (a parameter server, an evaluator):
    ``metrics/<node>`` plus a registry the master's plan loop reads besides the members."""
    kv.set(f"metrics/{node}", json.dumps(m))
    reg = set((kv.get_str("metrics/extra_nodes") or "").split(","))
    if node not in reg:
        kv.append("metrics/extra_nodes", node + ",")
