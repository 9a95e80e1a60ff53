"""Row-sparse embedding tables served by the parameter servers.

CTR models (the reference's example job is ``elastic-deepctr-job``,
docs/design/elastic-training-operator.md:35) are dominated by embedding
tables that are far larger than what one step touches.  A
:class:`PSEmbedding` therefore never holds its table on a worker once it is
bound to a :class:`~easydl_amd.ps.client.PSClient`:

* forward: ``unique(ids)`` -> pull only those rows from their owning PS
  (rows are striped: global row ``r`` lives on PS ``r % num_ps`` at local row
  ``r // num_ps``, so every shard gets a uniform share of hot ids) -> a leaf
  ``[n_unique, dim]`` tensor -> ``F.embedding(inverse, rows)``;
* backward: autograd leaves the already de-duplicated row gradients on that
  leaf; :meth:`take_grads` hands ``(unique ids, grads)`` to the client's push;
* the PS applies a lazy (touched-rows-only) AdamW / Adagrad / SGD
  (csrc/kernels/ps_sparse.hip when the shard lives on a GPU).

Unbound (no PS: unit tests, single-process runs) it is a plain dense
embedding with a local ``weight`` parameter.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import nn


class PSEmbedding(nn.Module):
    def __init__(self, num_rows: int, dim: int, init_std: float = 0.01, device=None):
        super().__init__()
        if dim % 4:
            raise ValueError("PSEmbedding dim must be a multiple of 4 (16-byte rows for the HIP kernels)")
        self.num_rows, self.dim, self.init_std = int(num_rows), int(dim), float(init_std)
        self.weight = nn.Parameter(torch.randn(num_rows, dim, device=device) * init_std)
        self._client = None
        self._name = None
        self._pending: list[tuple[torch.Tensor, torch.Tensor]] = []

    @property
    def bound(self) -> bool:
        return self._client is not None

    def attach(self, client, name: str) -> None:
        """Serve rows from the PS shards from now on (drops the local table)."""
        self._client, self._name = client, name
        self.weight = None

    def forward(self, ids: torch.Tensor) -> torch.Tensor:
        if self._client is None:
            return F.embedding(ids, self.weight)
        uniq, inv = torch.unique(ids.reshape(-1), return_inverse=True)
        rows = self._client.pull_rows(self._name, uniq).to(ids.device)
        if self.training and torch.is_grad_enabled():
            rows.requires_grad_(True)
            self._pending.append((uniq, rows))
        return F.embedding(inv.view(ids.shape), rows)

    def take_grads(self) -> tuple[torch.Tensor, torch.Tensor] | None:
        """(unique ids, fp32 row grads) accumulated since the last call, or None."""
        items = [(u, r.grad) for u, r in self._pending if r.grad is not None]
        self._pending = []
        if not items:
            return None
        if len(items) == 1:
            return items[0][0], items[0][1].float()
        ids = torch.cat([u for u, _ in items])
        grads = torch.cat([g.float() for _, g in items])
        uniq, inv = torch.unique(ids, return_inverse=True)
        out = torch.zeros(uniq.numel(), self.dim, dtype=torch.float32, device=grads.device)
        out.index_add_(0, inv, grads)
        return uniq, out


def tables_of(model: nn.Module) -> dict[str, PSEmbedding]:
    return {n: m for n, m in model.named_modules() if isinstance(m, PSEmbedding)}


def table_shard_spec(model: nn.Module, num_ps: int, index: int) -> dict[str, dict]:
    """Per-table local row count / dim / init of PS ``index`` (row striping ``r % num_ps``)."""
    out = {}
    for n, m in tables_of(model).items():
        out[n] = {"rows": max(0, (m.num_rows - index + num_ps - 1) // num_ps), "dim": m.dim,
                  "init_std": m.init_std, "global_rows": m.num_rows}
    return out
