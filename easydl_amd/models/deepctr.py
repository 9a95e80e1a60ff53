"""DeepFM click-through-rate model with PS-served embedding tables.

The reference's only example job is a CTR job (``elastic-deepctr-job``,
``model_zoo.iris.dnn_estimator``; docs/design/elastic-training-operator.md:35-37),
i.e. the parameter-server workload EasyDL/ElasticDL were built for: huge,
row-sparse embedding tables plus a small dense network.  This is DeepFM
(Guo et al. 2017) in that shape:

* ``n_sparse`` categorical fields share ONE :class:`PSEmbedding` (field ``f``'s
  ids are offset by ``f * vocab``) of dim ``emb_dim`` for the FM / DNN part and
  one of dim 4 whose first column is the first-order weight;
* FM 2nd order: ``0.5 * sum_k((sum_f e_fk)^2 - sum_f e_fk^2)``;
* DNN over ``concat(e_1..e_F, dense)``;
* logit = linear + FM + DNN, binary cross-entropy.

:class:`SyntheticCTR` draws Zipf-skewed ids (hot rows, like real click logs)
and labels from a hidden FM-like teacher, so AUC/accuracy are meaningful
end-to-end signals without any dataset download.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import nn

from easydl_amd.ps.embedding import PSEmbedding


class DeepFM(nn.Module):
    def __init__(self, n_sparse: int = 26, n_dense: int = 13, vocab: int = 10000, emb_dim: int = 16,
                 hidden=(400, 400, 400), device=None):
        super().__init__()
        self.n_sparse, self.n_dense, self.vocab, self.emb_dim = n_sparse, n_dense, vocab, emb_dim
        self.emb = PSEmbedding(n_sparse * vocab, emb_dim, init_std=0.01, device=device)
        self.lin_emb = PSEmbedding(n_sparse * vocab, 4, init_std=0.0, device=device)
        self.dense_lin = nn.Linear(n_dense, 1, device=device)
        dims = [n_sparse * emb_dim + n_dense, *hidden]
        self.mlp = nn.ModuleList(nn.Linear(a, b, device=device) for a, b in zip(dims[:-1], dims[1:]))
        self.out = nn.Linear(dims[-1], 1, device=device)
        self.register_buffer("offsets", torch.arange(n_sparse, device=device) * vocab, persistent=False)

    def logits(self, sparse_ids: torch.Tensor, dense: torch.Tensor) -> torch.Tensor:
        ids = sparse_ids + self.offsets                     # [B, F] global rows
        e = self.emb(ids)                                   # [B, F, D]
        first = self.lin_emb(ids)[..., 0].sum(1) + self.dense_lin(dense).squeeze(1)
        s = e.sum(1)
        fm = 0.5 * (s * s - (e * e).sum(1)).sum(1)
        h = torch.cat([e.flatten(1), dense], 1)
        for layer in self.mlp:
            h = F.relu(layer(h))
        return first + fm + self.out(h).squeeze(1)

    def forward(self, sparse_ids, dense, label=None):
        z = self.logits(sparse_ids, dense)
        if label is None:
            return z
        return F.binary_cross_entropy_with_logits(z, label.float())


class SyntheticCTR:
    """Deterministic click log: Zipf(1.1) ids per field, 13 dense features, teacher labels."""

    def __init__(self, n: int = 100000, n_sparse: int = 26, n_dense: int = 13, vocab: int = 10000, seed: int = 0):
        self.n, self.n_sparse, self.n_dense, self.vocab, self.seed = n, n_sparse, n_dense, vocab, seed
        g = torch.Generator().manual_seed(seed)
        ranks = torch.arange(1, vocab + 1, dtype=torch.float64)
        self.p = (ranks ** -1.1) / (ranks ** -1.1).sum()
        self.t_emb = torch.randn(n_sparse, vocab, 4, generator=g) * 0.7
        self.t_dense = torch.randn(n_dense, generator=g) * 0.5

    def __len__(self):
        return self.n

    def batch(self, idx, device="cpu"):
        idx = list(idx)
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + (idx[0] if idx else 0))
        b = len(idx)
        ids = torch.multinomial(self.p.float(), b * self.n_sparse, replacement=True, generator=g)
        ids = ids.view(b, self.n_sparse)
        dense = torch.randn(b, self.n_dense, generator=g)
        te = self.t_emb[torch.arange(self.n_sparse).unsqueeze(0), ids]          # [B, F, 4]
        s = te.sum(1)
        z = 0.5 * (s * s - (te * te).sum(1)).sum(1) / self.n_sparse + dense @ self.t_dense + te[..., 0].sum(1) * 0.3
        y = (torch.rand(b, generator=g) < torch.sigmoid(z)).float()
        return ids.to(device), dense.to(device), y.to(device)


def auc(model: nn.Module, data: SyntheticCTR, n: int = 4000, device="cpu") -> float:
    """Rank-based ROC AUC on the last ``n`` samples."""
    with torch.no_grad():
        was = model.training
        model.eval()
        ids, dense, y = data.batch(range(data.n - n, data.n), device)
        z = model(ids, dense).float().cpu()
        model.train(was)
    y = y.cpu()
    order = torch.argsort(z)
    r = torch.empty_like(z)
    r[order] = torch.arange(1, len(z) + 1, dtype=z.dtype)
    pos = y.sum()
    neg = len(y) - pos
    if pos == 0 or neg == 0:
        return 0.5
    return float((r[y == 1].sum() - pos * (pos + 1) / 2) / (pos * neg))
