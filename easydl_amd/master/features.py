"""Job feature extraction for the Brain (reference
docs/design/elastic-training-operator.md:105-107: the trainer "extracts
features from the job" before asking the Brain for startup resources).

The trainer master reads the model description from the job (``spec.features``
hints or the ``EDL_MODEL`` / ``EDL_SEQ`` / ``EDL_MBS`` / ``EDL_ACCUM`` /
``EDL_TP`` environment the job passes to its workers), instantiates the model
on PyTorch's ``meta`` device — shapes only, no memory, no GPU — and derives:

* ``params`` and per-parameter state bytes (bf16 weights + fp32 master/m/v +
  bf16 grads = 16 B under mixed-precision AdamW, 12 B for fp32 SGD+momentum);
* ``flops_per_sample`` / ``tokens_per_step_per_rank``;
* ``activation_gb_per_rank`` (flash-attention transformer: S*b*d*(10 + 24/tp)
  bytes per layer without recomputation, Korthikanti et al. 2022; CNN: an
  approximate per-image footprint);
* ``state_gb_per_rank`` = params x bytes / tp, which the Brain compares with
  the 288 GB of HBM when it sizes TP, CU/HBM shares and snapshot intervals.

User-declared ``spec.features`` always win over extracted values.
"""
from __future__ import annotations

import logging

import torch

log = logging.getLogger(__name__)


def _param_count(model: torch.nn.Module) -> int:
    return sum(p.numel() for p in model.parameters())


def _llama(name: str, seq: int, mbs: int, tp: int) -> dict:
    from easydl_amd.models.llama import Llama, get_config
    cfg = get_config(name)
    with torch.device("meta"):
        n = _param_count(Llama(cfg, device="meta", dtype=torch.bfloat16))
    # bytes per layer: S*b*d*(10 + 24/tp) with flash attention and no sequence parallelism
    act = seq * mbs * cfg.dim * cfg.n_layers * (10.0 + 24.0 / tp) / 1e9
    return {"family": "llama", "params": float(n), "bytes_per_param_state": 16.0,
            "flops_per_sample": cfg.flops_per_token(seq) * seq, "tokens_per_step_per_rank": float(seq * mbs),
            "activation_gb_per_rank": round(act, 2), "seq": seq}


def _resnet(mbs: int) -> dict:
    from easydl_amd.models.resnet import resnet50
    with torch.device("meta"):
        n = _param_count(resnet50())
    # ~4.1 GFLOPs fwd per 224^2 image, x3 for training; activations ~100 MB/image in bf16
    return {"family": "resnet", "params": float(n), "bytes_per_param_state": 12.0, "flops_per_sample": 12.3e9,
            "activation_gb_per_rank": round(0.1 * mbs, 2)}


def _bert(name: str, seq: int, mbs: int) -> dict:
    from easydl_amd.models.bert import BERT_LARGE, BERT_TINY, BertMLM
    cfg = BERT_TINY if "tiny" in name else BERT_LARGE
    with torch.device("meta"):
        n = _param_count(BertMLM(cfg))
    act = 34.0 * seq * mbs * cfg.dim * cfg.n_layers / 1e9
    return {"family": "bert", "params": float(n), "bytes_per_param_state": 16.0, "flops_per_sample": 6.0 * n * seq,
            "tokens_per_step_per_rank": float(seq * mbs), "activation_gb_per_rank": round(act, 2), "seq": seq}


def extract(job) -> dict:
    """Features of an :class:`~easydl_amd.api.spec.ElasticJob` (never raises)."""
    hints = dict(job.features or {})
    env = dict(job.env or {})
    name = str(hints.get("model") or env.get("EDL_MODEL") or "")
    seq = int(hints.get("seq") or env.get("EDL_SEQ") or 8192)
    mbs = int(hints.get("mbs") or env.get("EDL_MBS") or 1)
    accum = int(hints.get("accum") or env.get("EDL_ACCUM") or 1)
    tp = int(hints.get("tp") or env.get("EDL_TP") or 1)
    out: dict = {"mode": job.mode, "min_workers": job.min_workers, "max_workers": job.max_workers, "tp": tp}
    try:
        if name.startswith("llama"):
            out.update(_llama(name, seq, mbs, tp))
        elif name.startswith("resnet"):
            out.update(_resnet(mbs))
        elif name.startswith("bert"):
            out.update(_bert(name, min(seq, 512), mbs))
        elif name:
            log.info("features: unknown model family %r, using declared hints only", name)
    except Exception as e:  # noqa: BLE001 - a bad hint must not stop the job
        log.warning("features: extraction for %r failed: %s", name, e)
    if "params" in out:
        out["state_gb_per_rank"] = round(out["params"] * out["bytes_per_param_state"] / tp / 1e9, 2)
        out["samples_per_step_per_rank"] = mbs * accum
    out.update(hints)  # the user's declarations win
    return out
