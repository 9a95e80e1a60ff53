"""BERT-large encoder with an MLM head (BASELINE.json config 4: "BERT-large async
PS, 2 PS + 6 workers"): 24 layers, d 1024, 16 heads, FFN 4096, vocab 30522.

Post-LN blocks exactly as BERT, with the residual add fused into the HIP
LayerNorm kernel (``add_layernorm``) and the MLM loss through the fused
cross-entropy kernel (logits padded to a multiple of 8 columns by the tied
decoder).  Attention (head_dim 64, bidirectional) runs through SDPA.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch
import torch.nn as nn
import torch.nn.functional as F

from easydl_amd.ops import fused, gradsink, norms
from easydl_amd.ops.attention import packed_qkv_attention


@dataclass
class BertConfig:
    vocab_size: int = 30522
    dim: int = 1024
    n_layers: int = 24
    n_heads: int = 16
    ffn_dim: int = 4096
    max_pos: int = 512
    eps: float = 1e-12
    init_std: float = 0.02

    @property
    def padded_vocab(self) -> int:
        return (self.vocab_size + 63) // 64 * 64


BERT_LARGE = BertConfig()
# EDL_RESGRAD=0: autograd sums each layer input's two gradients (A/B switch)
_RESGRAD = os.environ.get("EDL_RESGRAD", "1") != "0"
BERT_TINY = BertConfig(vocab_size=512, dim=64, n_layers=2, n_heads=4, ffn_dim=128, max_pos=64)


def _p(shape, std, device, dtype):
    t = torch.empty(shape, device=device, dtype=dtype)
    if std == 0:
        t.zero_()
    elif std == 1:
        t.fill_(1.0)
    else:
        t.normal_(0, std)
    return nn.Parameter(t)


class BertLayer(nn.Module):
    def __init__(self, c: BertConfig, device, dtype):
        super().__init__()
        d = c.dim
        self.c = c
        self.wqkv = _p((3 * d, d), c.init_std, device, dtype)
        self.bqkv = _p((3 * d,), 0, device, dtype)
        self.wo = _p((d, d), c.init_std, device, dtype)
        self.bo = _p((d,), 0, device, dtype)
        self.ln1_w = _p((d,), 1, device, dtype)
        self.ln1_b = _p((d,), 0, device, dtype)
        self.w1 = _p((c.ffn_dim, d), c.init_std, device, dtype)
        self.b1 = _p((c.ffn_dim,), 0, device, dtype)
        self.w2 = _p((d, c.ffn_dim), c.init_std, device, dtype)
        self.b2 = _p((d,), 0, device, dtype)
        self.ln2_w = _p((d,), 1, device, dtype)
        self.ln2_b = _p((d,), 0, device, dtype)

    def forward(self, x, B, S, mask=None):
        c = self.c
        H, hd = c.n_heads, c.dim // c.n_heads
        # x's two gradients (qkv input gradient + LN1's residual gradient) meet in the qkv
        # GEMM's epilogue instead of an add kernel (gradsink.ResidualGrad); same for the MLP
        r1, r2 = (gradsink.ResidualGrad(), gradsink.ResidualGrad()) if _RESGRAD else (None, None)
        qkv = fused.linear(x, self.wqkv, self.bqkv, res_grad=r1)
        if qkv.is_cuda and mask is None:
            # HIP kernels, head dim 64; dq / dk / dv land in one packed qkv gradient
            o = packed_qkv_attention(qkv, B, S, H, causal=False)
        else:
            q, k, v = (t.transpose(1, 2) for t in qkv.view(B, S, 3, H, hd).unbind(2))
            if q.is_cuda:
                o = F.scaled_dot_product_attention(q, k, v, attn_mask=mask)
            else:
                o = F.scaled_dot_product_attention(q.float(), k.float(), v.float(), attn_mask=mask).to(q.dtype)
            o = o.transpose(1, 2).reshape(B * S, c.dim)
        a = fused.linear(o, self.wo, self.bo)
        x, _ = norms.add_layernorm(a, x, self.ln1_w, self.ln1_b, c.eps, res_grad=r1)
        m = fused.gelu_mlp(x, self.w1, self.b1, self.w2, self.b2, res_grad=r2)
        x, _ = norms.add_layernorm(m, x, self.ln2_w, self.ln2_b, c.eps, res_grad=r2)
        return x


class BertMLM(nn.Module):
    def __init__(self, c: BertConfig = BERT_LARGE, device=None, dtype=torch.bfloat16):
        super().__init__()
        self.c = c
        d = c.dim
        self.tok = _p((c.padded_vocab, d), c.init_std, device, dtype)
        self.pos = _p((c.max_pos, d), c.init_std, device, dtype)
        self.typ = _p((2, d), c.init_std, device, dtype)
        self.ln_e_w = _p((d,), 1, device, dtype)
        self.ln_e_b = _p((d,), 0, device, dtype)
        self.layers = nn.ModuleList(BertLayer(c, device, dtype) for _ in range(c.n_layers))
        self.head_w = _p((d, d), c.init_std, device, dtype)
        self.head_b = _p((d,), 0, device, dtype)
        self.head_ln_w = _p((d,), 1, device, dtype)
        self.head_ln_b = _p((d,), 0, device, dtype)

    def forward(self, ids, labels=None):
        B, S = ids.shape
        c = self.c
        pos = torch.arange(S, device=ids.device)
        x = fused.embedding(ids.reshape(-1), self.tok) + self.pos[pos].repeat(B, 1) + self.typ[0]
        x = norms.layernorm(x, self.ln_e_w, self.ln_e_b, c.eps)
        for layer in self.layers:
            x = layer(x, B, S)
        h = F.gelu(fused.linear(x, self.head_w, self.head_b), approximate="tanh")
        h = norms.layernorm(h, self.head_ln_w, self.head_ln_b, c.eps)
        logits = fused.linear(h, self.tok)  # tied decoder, padded vocab
        if labels is None:
            return logits.view(B, S, -1)[..., :c.vocab_size]
        return fused.cross_entropy(logits, labels.reshape(-1))


class SyntheticMLM:
    """Masked-LM samples: 15 % of positions carry a label, the rest are ignored (-100)."""

    def __init__(self, vocab: int, seq: int, n: int = 1 << 30):
        self.vocab, self.seq, self.n = vocab, seq, n

    def __len__(self):
        return self.n

    def batch(self, idx, device="cpu"):
        idx = list(idx)
        g = torch.Generator(device=device).manual_seed(int(idx[0]) if idx else 0)
        ids = torch.randint(0, self.vocab, (len(idx), self.seq), device=device, generator=g)
        sel = torch.rand(len(idx), self.seq, device=device, generator=g) < 0.15
        labels = torch.where(sel, ids, torch.full_like(ids, -100))
        ids = torch.where(sel, torch.full_like(ids, 103), ids)  # [MASK]
        return ids, labels
