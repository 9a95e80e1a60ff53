"""Apply the Brain's per-rank resource plan inside a training process
(SURVEY.md §2.4 N12, B30):

* ``EDL_CU_MASK`` (hex over 256 CUs, set by the operator from ``resource.cu``)
  -> the process's compute stream is created CU-masked through the native
  runtime and made PyTorch's current stream (ExternalStream), so every kernel
  of this rank — GEMMs, our HIP kernels — runs only on its CU share;
* ``EDL_HBM_GB`` -> caching-allocator cap via ``set_per_process_memory_fraction``;
* CPU affinity is applied by the supervisor at spawn time.
"""
from __future__ import annotations

import ctypes
import logging

import torch

from easydl_amd import _native

log = logging.getLogger(__name__)


def mask_words(hex_mask: str, ncu: int = 256) -> list[int]:
    v = int(hex_mask, 16)
    return [(v >> (32 * i)) & 0xFFFFFFFF for i in range((ncu + 31) // 32)]


def apply_cu_mask(device: torch.device, hex_mask: str):
    """Create a CU-masked stream and make it current; returns the ExternalStream."""
    rt = _native.runtime()
    words = mask_words(hex_mask)
    arr = (ctypes.c_uint32 * len(words))(*words)
    h = rt("edl_stream_create_cumask", device.index or 0, arr, len(words), 0)
    if not h:
        log.warning("CU mask %s could not be applied", hex_mask)
        return None
    s = torch.cuda.ExternalStream(h, device=device)
    torch.cuda.set_stream(s)
    return s


def apply_hbm_cap(device: torch.device, hbm_gb: float) -> float:
    total = torch.cuda.get_device_properties(device).total_memory / 2**30
    frac = max(0.01, min(1.0, hbm_gb / total))
    torch.cuda.set_per_process_memory_fraction(frac, device)
    return frac


def apply_plan(ctx, device: torch.device) -> dict:
    out = {}
    if device.type != "cuda":
        return out
    if ctx.cu_mask:
        out["cu_stream"] = apply_cu_mask(device, ctx.cu_mask) is not None
        out["cu_count"] = bin(int(ctx.cu_mask, 16)).count("1")
    if ctx.hbm_gb:
        out["hbm_fraction"] = apply_hbm_cap(device, ctx.hbm_gb)
    return out
