"""Row-sparse parameter-server ops (csrc/kernels/ps_sparse.hip).

* :func:`embed_gather`        rows of an fp32 table -> fp32/bf16 [n, dim] (PS pull)
* :func:`segment_sum_rows`    duplicate ids -> (unique ids, compact fp32 grad) (PS push)
* :func:`sparse_rows_update`  lazy AdamW / Adagrad / SGD on the touched rows only
* :func:`pull_cast`           fp32 shard -> bf16 worker copy (dense pull)

GPU tensors run the HIP kernels; CPU tensors run the same math in PyTorch
(that is the CPU/gloo PS path and the numerics reference of the GPU tests).
Out-of-range ids gather a zero row and are dropped on scatter, on both paths.
"""
from __future__ import annotations

import math

import torch

from easydl_amd import _native

OPT_KIND = {"adam": 0, "adamw": 0, "adagrad": 1, "sgd": 2}


def _check_rows(table: torch.Tensor) -> None:
    if table.dim() != 2 or table.dtype != torch.float32 or not table.is_contiguous() or table.shape[1] % 4:
        raise ValueError("embedding tables are contiguous fp32 [rows, dim] with dim % 4 == 0")


def embed_gather(table: torch.Tensor, ids: torch.Tensor, out_dtype=torch.float32) -> torch.Tensor:
    _check_rows(table)
    ids = ids.reshape(-1).to(torch.int64)
    rows, dim = table.shape
    if _native.use_hip(table):
        ids = ids.to(table.device).contiguous()
        out = torch.empty(ids.numel(), dim, dtype=out_dtype, device=table.device)
        _native.kernels().check("edl_embed_gather", table.data_ptr(), ids.data_ptr(), ids.numel(), dim, rows,
                                out.data_ptr(), 1 if out_dtype == torch.bfloat16 else 0,
                                _native.stream_of(table))
        return out
    ok = (ids >= 0) & (ids < rows)
    out = table[ids.clamp(0, rows - 1)] * ok.unsqueeze(1)
    return out.to(out_dtype)


def scatter_add_rows(acc: torch.Tensor, ids: torch.Tensor, grad: torch.Tensor) -> torch.Tensor:
    """acc[ids[i]] += grad[i] (duplicates accumulate; out-of-range ids are dropped)."""
    _check_rows(acc)
    ids = ids.reshape(-1).to(torch.int64)
    grad = grad.reshape(ids.numel(), acc.shape[1])
    if _native.use_hip(acc):
        ids = ids.to(acc.device).contiguous()
        grad = grad.to(acc.device).contiguous()
        if grad.dtype not in (torch.float32, torch.bfloat16):
            grad = grad.float()
        _native.kernels().check("edl_embed_scatter_add", acc.data_ptr(), ids.data_ptr(), grad.data_ptr(),
                                1 if grad.dtype == torch.bfloat16 else 0, ids.numel(), acc.shape[1], acc.shape[0],
                                _native.stream_of(acc))
        return acc
    ok = (ids >= 0) & (ids < acc.shape[0])
    acc.index_add_(0, ids[ok], grad[ok].float())
    return acc


def segment_sum_rows(ids: torch.Tensor, grad: torch.Tensor, rows: int) -> tuple[torch.Tensor, torch.Tensor]:
    """(unique valid ids, fp32 [n_unique, dim] sums of their gradient rows)."""
    ids = ids.reshape(-1).to(torch.int64)
    dim = grad.shape[-1]
    grad = grad.reshape(ids.numel(), dim)
    ok = (ids >= 0) & (ids < rows)
    if not bool(ok.all()):
        ids, grad = ids[ok], grad[ok]
    uniq, inv = torch.unique(ids, return_inverse=True)
    compact = torch.zeros(uniq.numel(), dim, dtype=torch.float32, device=grad.device)
    if uniq.numel():
        scatter_add_rows(compact, inv, grad)
    return uniq, compact


def sparse_rows_update(w: torch.Tensor, m: torch.Tensor | None, v: torch.Tensor | None, uniq: torch.Tensor,
                       grad: torch.Tensor, *, kind: str = "adam", lr: float, beta1: float = 0.9,
                       beta2: float = 0.999, eps: float = 1e-8, weight_decay: float = 0.0, step: int = 1,
                       scale: float = 1.0) -> None:
    """Lazy optimizer update of rows ``uniq`` (unique ids) with ``grad[i]`` for ``uniq[i]``."""
    _check_rows(w)
    k = OPT_KIND[kind]
    if _native.use_hip(w):
        _native.kernels().check("edl_sparse_rows_update", w.data_ptr(), _native.ptr(m), _native.ptr(v),
                                uniq.data_ptr(), grad.contiguous().data_ptr(), uniq.numel(), w.shape[1], w.shape[0],
                                k, lr, beta1, beta2, eps, weight_decay, int(step), float(scale),
                                _native.stream_of(w))
        return
    if uniq.numel() == 0:
        return
    g = grad.float() * scale
    p = w[uniq]
    decay = 1.0 - lr * weight_decay
    if k == 0:
        mm = m[uniq].mul_(beta1).add_(g, alpha=1 - beta1)
        vv = v[uniq].mul_(beta2).addcmul_(g, g, value=1 - beta2)
        denom = vv.sqrt() / math.sqrt(1 - beta2 ** step) + eps
        p = p * decay - (lr / (1 - beta1 ** step)) * mm / denom
        m[uniq], v[uniq] = mm, vv
    elif k == 1:
        vv = v[uniq] + g * g
        p = p * decay - lr * g / (vv.sqrt() + eps)
        v[uniq] = vv
    else:
        p = p * decay - lr * g
    w[uniq] = p


def pull_cast(src: torch.Tensor, dst: torch.Tensor) -> torch.Tensor:
    """dst (bf16) <- src (fp32); the src pointer may be an IPC-mapped peer shard."""
    if dst.is_cuda:
        if src.numel() != dst.numel() or src.numel() % 8:
            raise ValueError("pull_cast: equal sizes, multiple of 8 elements")
        _native.kernels().check("edl_ps_pull_cast", src.data_ptr(), dst.data_ptr(), src.numel(),
                                _native.stream_of(dst))
        return dst
    dst.copy_(src)
    return dst


class MultiCopyPlan:
    """One-launch dense push / pull between a worker's scattered parameter (or
    gradient) tensors and a PS's flat fp32 buffer (``edl_ps_multi_copy``,
    csrc/kernels/ps_sparse.hip).  ``items`` = [(tensor or None, flat offset, numel)];
    None pushes zeros (a parameter without a gradient).  The tensor table lives in
    device memory; :attr:`key` (the tensors' data pointers) tells the caller when
    it must be rebuilt."""

    def __init__(self, items, device):
        k = _native.kernels()
        chunk = k("edl_ps_multi_chunk")
        rows, bstart = [], [0]
        ptrs = []
        for t, off, n in items:
            if off % 4:
                raise ValueError("MultiCopyPlan: PS offsets must be multiples of 4 elements")
            if t is None:
                kind, ptr = 2, 0
            else:
                if not t.is_contiguous() or t.numel() != n or t.dtype not in (torch.float32, torch.bfloat16):
                    raise ValueError("MultiCopyPlan: contiguous fp32 / bf16 tensors of the layout's size")
                kind, ptr = (1 if t.dtype == torch.bfloat16 else 0), t.data_ptr()
                if ptr % (8 if kind == 1 else 16):
                    raise ValueError("MultiCopyPlan: misaligned tensor")
            ptrs.append(ptr)
            rows.append([ptr, off, n, kind])
            bstart.append(bstart[-1] + -(-n // chunk))
        self.n = len(rows)
        self.nblocks = bstart[-1]
        self.table = torch.tensor(rows, dtype=torch.int64).to(device)
        self.bstart = torch.tensor(bstart, dtype=torch.int64).to(device)
        self.key = tuple(ptrs)

    def run(self, flat_ptr: int, push: bool, stream=None) -> None:
        s = stream if stream is not None else torch.cuda.current_stream(self.table.device).cuda_stream
        _native.kernels().check("edl_ps_multi_copy", self.table.data_ptr(), self.bstart.data_ptr(), self.n,
                                self.nblocks, flat_ptr, 1 if push else 0, s)


def ptr_array(tensors_or_ptrs, device) -> torch.Tensor:
    """Device int64 array of pointers (the kernels' per-PS tables)."""
    vals = [t if isinstance(t, int) else t.data_ptr() for t in tensors_or_ptrs]
    return torch.tensor(vals, dtype=torch.int64).to(device)


def embed_gather_striped(tabs: torch.Tensor, nrows: torch.Tensor, ids: torch.Tensor, dim: int,
                         out_dtype=torch.float32) -> torch.Tensor:
    """Rows ``ids`` (global) of a table striped over ``P = len(tabs)`` PS stripes (row r at
    local row r // P of stripe r % P); ``tabs``/``nrows``: device int64 arrays of the
    (IPC-mapped) stripe pointers and their row counts.  One launch, no host sync."""
    ids = ids.reshape(-1).to(torch.int64).contiguous()
    out = torch.empty(ids.numel(), dim, dtype=out_dtype, device=ids.device)
    _native.kernels().check("edl_embed_gather_striped", tabs.data_ptr(), nrows.data_ptr(), tabs.numel(),
                            ids.data_ptr(), ids.numel(), dim, out.data_ptr(), 1 if out_dtype == torch.bfloat16 else 0,
                            _native.stream_of(ids))
    return out


def sparse_split_push(ids: torch.Tensor, grad: torch.Tensor, inbox_ids: torch.Tensor, inbox_grad: torch.Tensor,
                      inbox_cnt: torch.Tensor, cap: int, scratch: torch.Tensor) -> None:
    """Write unique global ``ids`` and their fp32 row ``grad`` into the owners' inboxes
    (device arrays of P peer pointers: local-id buffers, gradient buffers, int32 counts).
    ``scratch``: int32 [>= P] on ids' device."""
    ids = ids.reshape(-1).to(torch.int64).contiguous()
    grad = grad.float().contiguous()
    if ids.numel() > cap:
        raise ValueError(f"sparse push of {ids.numel()} rows exceeds the inbox capacity {cap}")
    _native.kernels().check("edl_sparse_split_push", ids.data_ptr(), grad.data_ptr(), ids.numel(), grad.shape[1],
                            inbox_ids.numel(), inbox_ids.data_ptr(), inbox_grad.data_ptr(), inbox_cnt.data_ptr(),
                            scratch.data_ptr(), int(cap), _native.stream_of(ids))


def sparse_inbox_update(w: torch.Tensor, m, v, ids: torch.Tensor, grad: torch.Tensor, count: torch.Tensor, *,
                        kind: str = "adam", lr: float, beta1: float = 0.9, beta2: float = 0.999, eps: float = 1e-8,
                        weight_decay: float = 0.0, step: int = 1, scale: float = 1.0) -> None:
    """Lazy optimizer update from a worker's sparse inbox; the row count is read on the
    device (``count``: int32, written by the worker's push)."""
    _check_rows(w)
    _native.kernels().check("edl_sparse_inbox_update", w.data_ptr(), _native.ptr(m), _native.ptr(v), ids.data_ptr(),
                            grad.data_ptr(), count.data_ptr(), ids.numel(), w.shape[1], w.shape[0], OPT_KIND[kind],
                            lr, beta1, beta2, eps, weight_decay, int(step), float(scale), _native.stream_of(w))


def ps_signal(flag: torch.Tensor, value: int, stream) -> None:
    """Stream-ordered system-scope store of ``value`` into ``flag`` (an IPC-mapped peer word)."""
    _native.kernels().check("edl_ps_signal", flag.data_ptr(), int(value) & 0xFFFFFFFF, stream.cuda_stream)


def ps_wait(flag: torch.Tensor, value: int, timeout_s: float, status: torch.Tensor, stream) -> None:
    """``stream`` waits (on the device, bounded) until ``flag`` >= ``value``; a give-up sets status[0]."""
    _native.kernels().check("edl_ps_wait", flag.data_ptr(), int(value) & 0xFFFFFFFF, float(timeout_s),
                            status.data_ptr(), stream.cuda_stream)
