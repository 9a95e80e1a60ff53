"""Which exceptions mean "a peer of this epoch is gone" (drop the step, re-form the
epoch) and which are bugs (raise).  Round 4 matched any RuntimeError whose text
contained "peer", "timed out", "connection", ... -- a genuine bug with such a word in
its message turned into a silent drop-and-reconfigure loop.  Now by type first:

* membership failures: :class:`CommAborted` (our watchdog aborted the epoch),
  :class:`XgmiAborted` (the xGMI engine's abort word is set; its other errors --
  misuse, a failed launch or IPC mapping -- are not membership failures),
  ``torch.distributed.DistBackendError`` / ``DistNetworkError`` (RCCL / c10d
  transport errors);
* gloo raises plain ``RuntimeError`` from its TCP transport, so only those whose
  text carries a gloo transport signature ("gloo/transport", "Connection closed by
  peer", "Connection reset by peer", "Timed out waiting ... for recv/send") count;
* everything else is NOT a membership failure: ``DistStoreError`` (the job
  master's store itself is broken: nothing to re-form with), ``ValueError``,
  shape errors, CUDA/HIP errors of our own kernels, ...
"""
from __future__ import annotations

import re

import torch.distributed as dist

_GLOO_TRANSPORT = re.compile(
    r"gloo/transport|connection closed by peer|connection reset by peer|"
    r"timed out waiting \d+ms for (recv|send)|nccl communicator was aborted|processgroupnccl.*abort",
    re.IGNORECASE)


def is_comm_error(e: BaseException) -> bool:
    from easydl_amd.parallel.comm import CommAborted
    from easydl_amd.parallel.xgmi import XgmiAborted
    if isinstance(e, (CommAborted, XgmiAborted)):
        return True
    store_err = getattr(dist, "DistStoreError", None)
    if store_err is not None and isinstance(e, store_err):
        return False
    typed = tuple(t for t in (getattr(dist, "DistBackendError", None), getattr(dist, "DistNetworkError", None))
                  if t is not None)
    if typed and isinstance(e, typed):
        return True
    return type(e) is RuntimeError and bool(_GLOO_TRANSPORT.search(str(e)))
