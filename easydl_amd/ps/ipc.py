"""GPU data plane of the parameter server on one node.

When a PS shard lives in HBM, bulk bytes never cross TCP: the PS exports its
fp32 parameter shard and one gradient inbox per worker as IPC handles
(dmabuf-backed, ``HSA_ENABLE_IPC_MODE_LEGACY=0``); a worker maps them once and

* **pull**: after a small TCP round trip that returns the shard version (and,
  in sync mode, waits for the wanted one), every parameter is copied out of
  the mapped shard by ``edl_ps_pull_cast`` (csrc/kernels/ps_sparse.hip) running
  on the WORKER's GPU — fp32 read over xGMI, cast, bf16 written locally — or a
  plain peer copy for fp32 models;
* **push**: the worker writes its gradients straight into its inbox in the PS's
  HBM (peer writes), synchronises its stream, then sends ``push_ipc``; the PS
  applies the fused AdamW kernel with the inbox AS the gradient (async) or
  adds it into the round accumulator (sync), and answers only after that
  kernel has finished reading the inbox, so the worker may overwrite it.

TCP keeps the control messages (versions, sparse rows, membership), so a PS
replacement is discovered exactly like the TCP transport (re-resolve,
re-open the handles of the new incarnation).
"""
from __future__ import annotations

import base64

import torch
from torch.multiprocessing.reductions import rebuild_cuda_tensor, reduce_tensor


def _b(x):
    return None if x is None else base64.b64encode(bytes(x)).decode()


def _u(x):
    return None if x is None else base64.b64decode(x)


def export_tensor(t: torch.Tensor) -> dict:
    """JSON-safe IPC description of a CUDA tensor (the producer keeps ``t`` alive)."""
    _, args = reduce_tensor(t)
    (_, size, stride, toff, _, dtype, dev, handle, ssize, soff, _, rch, rco, evh, evs) = args
    return {"size": list(size), "stride": list(stride), "toff": int(toff), "dtype": str(dtype).split(".")[-1],
            "device": int(dev), "handle": _b(handle), "ssize": int(ssize), "soff": int(soff), "rch": _b(rch),
            "rco": int(rco), "evh": _b(evh), "evs": bool(evs)}


def import_tensor(d: dict) -> torch.Tensor:
    return rebuild_cuda_tensor(torch.Tensor, torch.Size(d["size"]), tuple(d["stride"]), d["toff"],
                               torch.storage.TypedStorage, getattr(torch, d["dtype"]), d["device"], _u(d["handle"]),
                               d["ssize"], d["soff"], False, _u(d["rch"]), d["rco"], _u(d["evh"]), d["evs"])
