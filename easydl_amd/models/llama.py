"""Llama-3 family decoder (8B / 70B / small test configs), built on the fused ops.

Layout choices for MI355X:
* ONE fused QKV GEMM ([(H+2KV)*D, d] weight) and ONE fused gate+up GEMM
  ([2F, d]) — fewer, larger hipBLASLt calls (N = 6144 / 28672 at d = 4096);
* RoPE + QKV split in one HIP pass producing flash-attention's [B,S,H,D]
  layout; SwiGLU, residual-add+RMSNorm and the vocab-128256 cross-entropy
  are single HIP passes (csrc/kernels);
* every weight gradient is written straight into the flat gradient buffer;
* with 288 GB of HBM per GPU the 8B model trains at 8k context WITHOUT
  activation recompute (≈1.1 GB of saved activations per layer at 8k
  tokens); ``recompute=True`` is available for the 70B/TP configs.

Tensor-parallel variants (column/row sharded projections) are built by
:mod:`easydl_amd.parallel.tp` on top of the same block.
Capability source: BASELINE.json configs 3 and 5 (Llama-3 8B DDP, 70B TP=8).
"""
from __future__ import annotations

import math
from dataclasses import asdict, dataclass

import torch
import torch.nn as nn
import torch.nn.functional as F
import torch.utils.checkpoint as ckpt

from easydl_amd.ops import fused, norms
from easydl_amd.parallel.flat import await_update


@dataclass
class LlamaConfig:
    vocab_size: int = 128256
    dim: int = 4096
    n_layers: int = 32
    n_heads: int = 32
    n_kv_heads: int = 8
    ffn_dim: int = 14336
    rope_theta: float = 500000.0
    norm_eps: float = 1e-5
    max_seq_len: int = 8192
    rope_scaling: dict | None = None
    tie_embeddings: bool = False
    init_std: float = 0.02
    # True: every layer's activations are recomputed in the backward; an int r: the first r layers
    # only (a takeover short of HBM recomputes just enough of them, trainer/recovery.py)
    recompute: bool | int = False

    @property
    def head_dim(self) -> int:
        return self.dim // self.n_heads

    def num_params(self) -> int:
        d, f, v, L = self.dim, self.ffn_dim, self.vocab_size, self.n_layers
        hd = self.head_dim
        attn = d * (self.n_heads + 2 * self.n_kv_heads) * hd + self.n_heads * hd * d
        mlp = 3 * d * f
        per_layer = attn + mlp + 2 * d
        emb = v * d * (1 if self.tie_embeddings else 2)
        return L * per_layer + emb + d

    def matmul_params(self) -> int:
        """Parameters that take part in a GEMM per token (LM head included, embedding lookup excluded)."""
        d, f, L, hd = self.dim, self.ffn_dim, self.n_layers, self.head_dim
        attn = d * (self.n_heads + 2 * self.n_kv_heads) * hd + self.n_heads * hd * d
        return L * (attn + 3 * d * f) + self.vocab_size * d

    def flops_per_token(self, seq_len: int) -> float:
        """Training FLOPs/token: 6*N_matmul + causal attention fwd+bwd (6*L*S*d)."""
        return 6.0 * self.matmul_params() + 6.0 * self.n_layers * seq_len * self.dim

    def to_dict(self):
        return asdict(self)


CONFIGS = {
    "llama3-8b": LlamaConfig(),
    "llama3-70b": LlamaConfig(dim=8192, n_layers=80, n_heads=64, n_kv_heads=8, ffn_dim=28672),
    "llama3.2-1b": LlamaConfig(dim=2048, n_layers=16, n_heads=32, n_kv_heads=8, ffn_dim=8192, tie_embeddings=True),
    "llama-tiny": LlamaConfig(vocab_size=512, dim=128, n_layers=2, n_heads=4, n_kv_heads=2, ffn_dim=256,
                              max_seq_len=256),
    "llama-small": LlamaConfig(vocab_size=32000, dim=1024, n_layers=8, n_heads=16, n_kv_heads=4, ffn_dim=2816,
                               max_seq_len=2048),
}


def get_config(name: str, **overrides) -> LlamaConfig:
    import copy
    cfg = copy.deepcopy(CONFIGS[name])
    for k, v in overrides.items():
        setattr(cfg, k, v)
    return cfg


def _param(shape, std, device, dtype, init=True):
    t = torch.empty(shape, device=device, dtype=dtype)
    if init:
        if std == 0:
            t.fill_(1.0)
        else:
            t.normal_(0.0, std)
    return nn.Parameter(t)


def attention(q, k, v, causal=True):
    """q [B,H,S,D], k/v [B,KV,S,D] -> [B,H,S,D] (GQA).

    GPU: the hand-written kernels of csrc/kernels/attention.hip (default;
    1.4x / 1.8x faster than PyTorch SDPA's AOTriton forward / backward at the
    8k-context shape, profiles/r01_attention_kernels.md); ``EDL_ATTN=sdpa``
    selects SDPA for A/B runs."""
    H, KV = q.shape[1], k.shape[1]
    if q.is_cuda:
        import os
        if os.environ.get("EDL_ATTN", "hip") == "hip":
            from easydl_amd.ops.attention import flash_attention
            return flash_attention(q, k, v, causal=causal)
        return F.scaled_dot_product_attention(q, k, v, is_causal=causal, enable_gqa=(H != KV))
    if H != KV:
        k = k.repeat_interleave(H // KV, dim=1)
        v = v.repeat_interleave(H // KV, dim=1)
    return F.scaled_dot_product_attention(q.float(), k.float(), v.float(), is_causal=causal).to(q.dtype)


class LlamaBlock(nn.Module):
    def __init__(self, cfg: LlamaConfig, device=None, dtype=torch.bfloat16, n_heads=None, n_kv_heads=None,
                 ffn_dim=None):
        super().__init__()
        self.cfg = cfg
        self.n_heads = n_heads or cfg.n_heads
        self.n_kv = n_kv_heads or cfg.n_kv_heads
        self.ffn = ffn_dim or cfg.ffn_dim
        d, hd, std = cfg.dim, cfg.head_dim, cfg.init_std
        out_std = std / math.sqrt(2 * cfg.n_layers)
        self.attn_norm = _param((d,), 0, device, dtype)
        self.wqkv = _param(((self.n_heads + 2 * self.n_kv) * hd, d), std, device, dtype)
        self.wo = _param((d, self.n_heads * hd), out_std, device, dtype)
        self.mlp_norm = _param((d,), 0, device, dtype)
        self.w_gu = _param((2 * self.ffn, d), std, device, dtype)
        self.w_down = _param((d, self.ffn), out_std, device, dtype)
        # tensor-parallel hooks (identity for the dense model): tp_copy before the
        # column-parallel projections, tp_reduce after the row-parallel ones
        self.tp_reduce = None
        self.tp_copy = None
        # overlapped TP (parallel/tp.py): start(tensor) -> finish() all-reduce hooks used
        # inside the GEMM ops instead of tp_copy / tp_reduce
        self.tp_dx_reduce = None
        self.tp_out_reduce = None
        # sequence parallel: column-parallel weight gradients on the side stream, beside the
        # reduce-scatter of their input gradient
        self.tp_wgrad_side = False

    def _attn(self, n1, B, S, cos, sin):
        hd = self.cfg.head_dim
        if self.tp_copy is not None:
            n1 = self.tp_copy(n1)
        qkv = fused.linear(n1, self.wqkv, dx_reduce=self.tp_dx_reduce, wgrad_side=self.tp_wgrad_side)
        q, k, v = fused.rope_qkv(qkv, cos, sin, B, S, self.n_heads, self.n_kv, hd)
        o = attention(q, k, v, causal=True)
        o = o.transpose(1, 2).reshape(B * S, self.n_heads * hd)
        a = fused.linear(o, self.wo, out_reduce=self.tp_out_reduce)
        if self.tp_reduce is not None:
            a = self.tp_reduce(a)
        return a

    def _mlp(self, n2):
        if self.tp_copy is not None:
            n2 = self.tp_copy(n2)
        m = fused.swiglu_mlp(n2, self.w_gu, self.w_down, dx_reduce=self.tp_dx_reduce,
                             out_reduce=self.tp_out_reduce, wgrad_side=self.tp_wgrad_side)
        if self.tp_reduce is not None:
            m = self.tp_reduce(m)
        return m

    def forward(self, resid, delta, B, S, cos, sin):
        """resid: residual stream [B*S, d]; delta: previous block's output (added here)."""
        eps = self.cfg.norm_eps
        n1, s1 = norms.add_rmsnorm(delta, resid, self.attn_norm, eps) if delta is not None else \
            (norms.rmsnorm(resid, self.attn_norm, eps), resid)
        a = self._attn(n1, B, S, cos, sin)
        n2, s2 = norms.add_rmsnorm(a, s1, self.mlp_norm, eps)
        m = self._mlp(n2)
        return s2, m


class Llama(nn.Module):
    def __init__(self, cfg: LlamaConfig, device=None, dtype=torch.bfloat16):
        super().__init__()
        self.cfg = cfg
        self._edl_awaits_own = True   # hidden()/forward() await their direct parameters' updates
        d = cfg.dim
        self.embed = _param((cfg.vocab_size, d), cfg.init_std, device, dtype)
        self.layers = nn.ModuleList([LlamaBlock(cfg, device, dtype) for _ in range(cfg.n_layers)])
        self.norm = _param((d,), 0, device, dtype)
        self.lm_head = None if cfg.tie_embeddings else _param((cfg.vocab_size, d), cfg.init_std, device, dtype)
        self._rope = {}

    def rope(self, S, device):
        key = (S, str(device))
        if key not in self._rope:
            self._rope[key] = fused.rope_tables(max(S, 1), self.cfg.head_dim, self.cfg.rope_theta, device,
                                                self.cfg.rope_scaling)
        return self._rope[key]

    def hidden(self, ids):
        B, S = ids.shape
        cos, sin = self.rope(S, ids.device)
        await_update(self.embed)      # (its own parameters: see install_update_waits)
        x = fused.embedding(ids.reshape(-1), self.embed)
        resid, delta = x, None
        rc = self.cfg.recompute
        n_rc = len(self.layers) if rc is True else int(rc or 0)
        for i, layer in enumerate(self.layers):
            if i < n_rc and self.training:
                resid, delta = ckpt.checkpoint(layer, resid, delta, B, S, cos, sin, use_reentrant=False)
            else:
                resid, delta = layer(resid, delta, B, S, cos, sin)
        await_update(self.norm)
        n, _ = norms.add_rmsnorm(delta, resid, self.norm, self.cfg.norm_eps)
        return n

    def forward(self, ids, labels=None):
        n = self.hidden(ids)
        w = self.embed if self.lm_head is None else self.lm_head
        await_update(w)
        logits = fused.linear(n, w)
        if labels is None:
            return logits.view(*ids.shape, -1)
        return fused.cross_entropy(logits, labels.reshape(-1))
