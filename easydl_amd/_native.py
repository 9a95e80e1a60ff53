"""ctypes bindings for the in-tree native libraries.

``libedl_kernels.so`` (HIP, gfx950) and ``libedl_runtime.so`` (host C++) are
built by :mod:`easydl_amd._build` into ``easydl_amd/lib``.  Kernels take raw
device pointers plus the caller's current ``hipStream_t`` so every launch is
stream-ordered with PyTorch work and capturable in a HIP graph.

Policy: on a machine with a GPU the HIP path is mandatory.  If the library is
missing or fails to load, :func:`kernels` raises — there is no silent eager
fallback for CUDA tensors.  CPU tensors use the pure-PyTorch reference
implementations in :mod:`easydl_amd.ops` (that is what the CPU test tier runs).
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch

_LIBDIR = os.environ.get("EDL_LIBDIR") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib")
_lock = threading.Lock()
_kern = None
_rt = None

c_void_p = ctypes.c_void_p
c_int = ctypes.c_int
c_i64 = ctypes.c_int64
c_float = ctypes.c_float
c_fp = ctypes.POINTER(ctypes.c_float)

# name -> (argtypes); every kernel entry point returns int (hipError_t)
_KERNEL_SIGS = {
    "edl_adamw_flat": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_i64, c_float, c_float, c_float,
                       c_float, c_float, c_i64, c_float, c_void_p, c_void_p],
    "edl_adamw_flat_m16": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_i64, c_float, c_float,
                           c_float, c_float, c_float, c_i64, c_float, c_void_p, c_void_p],
    "edl_gemm_nt": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p],
    "edl_gemm_nt8": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p],
    "edl_gemm_nt_diag": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                         c_void_p],
    "edl_sgd_flat": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_i64, c_float, c_float, c_float, c_float,
                     c_void_p, c_void_p],
    "edl_sumsq_nparts": [c_i64],
    "edl_sumsq_partial": [c_void_p, c_int, c_i64, c_void_p, c_void_p],
    "edl_clip_finalize": [c_void_p, c_int, c_float, c_float, c_void_p, c_void_p],
    "edl_norm_max_cols": [],
    "edl_norm_bwd_groups": [c_int, c_int],
    "edl_rmsnorm_fwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_float, c_void_p],
    "edl_layernorm_fwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                          c_int, c_float, c_void_p],
    "edl_rmsnorm_bwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p],
    "edl_layernorm_bwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                          c_int, c_int, c_void_p],
    "edl_colsum": [c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_void_p],
    "edl_swiglu_fwd": [c_void_p, c_void_p, c_i64, c_int, c_void_p],
    "edl_swiglu_bwd": [c_void_p, c_void_p, c_void_p, c_i64, c_int, c_void_p],
    "edl_swiglu_fwd_t": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p],
    "edl_swiglu_bwd_t": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p],
    "edl_gelu_fwd_t": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p],
    "edl_qkv_split": [c_void_p, c_void_p, c_void_p, c_void_p, c_i64, c_int, c_void_p],
    "edl_gelu_bwd_t": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p],
    "edl_rope_qkv_fwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_i64, c_int, c_int, c_int,
                         c_int, c_void_p],
    "edl_rope_qkv_bwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_i64, c_int, c_int, c_int,
                         c_int, c_void_p],
    "edl_xent_fwd_bwd": [c_void_p, c_void_p, c_void_p, c_i64, c_int, c_i64, c_int, c_void_p, c_void_p, c_void_p],
    "edl_xent_grad_lse": [c_void_p, c_void_p, c_void_p, c_i64, c_int, c_i64, c_void_p, c_void_p],
    "edl_xent_vp": [c_void_p, c_void_p, c_void_p, c_i64, c_int, c_i64, c_i64, c_int, c_void_p, c_void_p],
    "edl_scale_bf16": [c_void_p, c_i64, c_void_p, c_float, c_void_p],
    "edl_transpose_bf16": [c_void_p, c_void_p, c_int, c_int, c_void_p],
    "edl_transpose_colsum_bf16": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p],
    "edl_transpose_tiles": [c_int],
    "edl_transpose_bf16_lds": [c_void_p, c_void_p, c_int, c_int, c_void_p],
    "edl_swiglu_fwd_t_lds": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p],
    "edl_swiglu_bwd_t_lds": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p],
    "edl_checksum": [c_void_p, c_i64, c_void_p, ctypes.c_uint64, c_void_p],
    "edl_attn_fwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int,
                     c_float, c_void_p],
    "edl_attn_bwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                     c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_float, c_void_p],
    "edl_transpose_bf16_multi": [c_void_p, c_int, c_int, c_void_p],
    "edl_attn_fwd_strided": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int,
                             c_int, c_float, c_i64, c_i64, c_void_p],
    "edl_attn_bwd_strided": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                             c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_float, c_i64,
                             c_i64, c_i64, c_void_p],
    "edl_attn_bwd_ws_bytes": (c_i64, [c_int, c_int, c_int, c_int, c_int]),
    "edl_xgmi_allreduce": [ctypes.POINTER(c_void_p), ctypes.POINTER(c_void_p), c_int, c_int, c_void_p, c_void_p,
                           c_i64, c_int, c_int, ctypes.c_uint32, c_int, c_void_p, ctypes.c_double, c_void_p,
                           c_void_p],
    "edl_xgmi_max_ranks": [],
    "edl_xgmi_allreduce_inplace": [ctypes.POINTER(c_void_p), ctypes.POINTER(c_void_p), c_int, c_int, c_i64, c_int,
                                   ctypes.c_uint32, c_int, c_void_p, ctypes.c_double, c_void_p, c_void_p],
    "edl_xgmi_barrier": [ctypes.POINTER(c_void_p), c_int, c_int, ctypes.c_uint32, c_void_p, ctypes.c_double, c_void_p,
                         c_void_p],
    "edl_xgmi_wallclock_hz": (c_i64, []),
    "edl_xgmi_pull_staged": [ctypes.POINTER(c_void_p), ctypes.POINTER(c_void_p), c_int, c_int, c_void_p, c_void_p,
                             c_i64, c_i64, ctypes.c_uint32, ctypes.c_uint32, c_int, c_void_p, ctypes.c_double, c_void_p,
                             c_void_p],
    "edl_xgmi_pull": [ctypes.POINTER(c_void_p), ctypes.POINTER(c_void_p), c_int, c_int, c_i64, ctypes.c_uint32,
                      ctypes.c_uint32, c_int, c_void_p, ctypes.c_double, c_void_p, c_void_p],
    "edl_xgmi_collective": [ctypes.POINTER(c_void_p), ctypes.POINTER(c_void_p), c_int, c_int, c_void_p, c_void_p,
                            c_i64, c_i64, c_int, c_int, ctypes.c_uint32, c_int, c_void_p, ctypes.c_double, c_void_p,
                            c_void_p],
    "edl_embed_gather": [c_void_p, c_void_p, c_i64, c_int, c_i64, c_void_p, c_int, c_void_p],
    "edl_embed_scatter_add": [c_void_p, c_void_p, c_void_p, c_int, c_i64, c_int, c_i64, c_void_p],
    "edl_sparse_rows_update": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_i64, c_int, c_i64, c_int, c_float,
                               c_float, c_float, c_float, c_float, c_i64, c_float, c_void_p],
    "edl_ps_pull_cast": [c_void_p, c_void_p, c_i64, c_void_p],
    "edl_ps_signal": [c_void_p, ctypes.c_uint32, c_void_p],
    "edl_ps_wait": [c_void_p, ctypes.c_uint32, ctypes.c_double, c_void_p, c_void_p],
    "edl_embed_gather_striped": [c_void_p, c_void_p, c_int, c_void_p, c_i64, c_int, c_void_p, c_int, c_void_p],
    "edl_sparse_split_push": [c_void_p, c_void_p, c_i64, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_i64,
                              c_void_p],
    "edl_sparse_inbox_update": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_i64, c_int, c_i64, c_int,
                                c_float, c_float, c_float, c_float, c_float, c_i64, c_float, c_void_p],
    "edl_ps_multi_chunk": [],
    "edl_ps_multi_copy": [c_void_p, c_void_p, c_int, c_i64, c_void_p, c_int, c_void_p],
    "edl_xgmi_max_blocks": [],
    "edl_diag_lds_dma": [c_void_p, c_void_p, c_int, c_void_p],
    "edl_gemm_tn_splits": [c_int, c_int, c_int],
    "edl_gemm_tn_ws_bytes": (c_i64, [c_int, c_int, c_int]),
    "edl_gemm_tn": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p],
    "edl_colsum_bf16_groups": [c_int],
    "edl_colsum_bf16_partial": [c_void_p, c_int, c_int, c_void_p, c_int, c_void_p],
    "edl_bn_groups": (c_int, [c_i64, c_int]),
    "edl_bn_fwd_train": [c_void_p] * 11 + [c_i64, c_int, c_float, c_float, c_int, c_void_p, c_void_p],
    "edl_bn_apply": [c_void_p] * 4 + [c_i64, c_int, c_int, c_void_p],
    "edl_bn_bwd": [c_void_p] * 14 + [c_i64, c_int, c_int, c_int, c_void_p],
}


class NativeError(RuntimeError):
    pass


class _Lib:
    def __init__(self, path: str, sigs: dict):
        self.path = path
        # torch is imported first (module top): its bundled libamdhip64.so.7 is then the
        # one HIP runtime of the process and our code objects register into it.
        self._h = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
        for name, sig in sigs.items():
            fn = getattr(self._h, name)
            if isinstance(sig, tuple):
                fn.restype, fn.argtypes = sig
            else:
                fn.argtypes = sig
                fn.restype = c_int
        self.sigs = sigs

    def raw(self, name):
        return getattr(self._h, name)

    def __call__(self, name: str, *args) -> int:
        rc = getattr(self._h, name)(*args)
        return rc

    def check(self, name: str, *args) -> None:
        rc = getattr(self._h, name)(*args)
        if rc != 0:
            raise NativeError(f"{name} failed with hipError {rc}")


def _load(path: str, sigs: dict) -> _Lib:
    if not os.path.exists(path):
        raise NativeError(
            f"native library {path} is missing: run `python -m easydl_amd._build` (or __graft_entry__.build())")
    return _Lib(path, sigs)


def kernels() -> _Lib:
    """The HIP kernel library; raises NativeError if it is not built."""
    global _kern
    if _kern is None:
        with _lock:
            if _kern is None:
                _kern = _load(os.path.join(_LIBDIR, "libedl_kernels.so"), _KERNEL_SIGS)
    return _kern


def kernels_available() -> bool:
    try:
        kernels()
        return True
    except (NativeError, OSError):
        return False


def runtime():
    """The host runtime library (supervisor, shm store, D2H engine)."""
    global _rt
    if _rt is None:
        with _lock:
            if _rt is None:
                from easydl_amd import _runtime_sigs
                _rt = _load(os.path.join(_LIBDIR, "libedl_runtime.so"), _runtime_sigs.SIGS)
    return _rt


def runtime_available() -> bool:
    try:
        runtime()
        return True
    except (NativeError, OSError):
        return False


def ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


def stream_of(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def use_hip(t: torch.Tensor) -> bool:
    """True when ``t`` lives on the GPU (then the HIP kernel MUST be used)."""
    return t.is_cuda
