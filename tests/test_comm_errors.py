"""Comm-failure classification by type and the watchdog's handling of
a job master that stops answering (it used to swallow every exception)."""
import time

import pytest
import torch
import torch.distributed as dist

from easydl_amd.parallel.comm import CommAborted, LocalCommunicator
from easydl_amd.parallel.errors import is_comm_error
from easydl_amd.parallel.xgmi import XgmiAborted, XgmiError
from easydl_amd.trainer.context import TrainerContext
from easydl_amd.trainer.elastic import ElasticTrainer, MasterUnreachable


@pytest.mark.parametrize("exc,expect", [
    (CommAborted("epoch 3 aborted"), True),
    (XgmiAborted("aborted"), True),
    (dist.DistBackendError("NCCL error in: ProcessGroupNCCL.cpp: remote process exited"), True),
    (dist.DistNetworkError("connection refused"), True),
    # gloo's TCP transport raises plain RuntimeError (measured on this torch: a peer's SIGKILL)
    (RuntimeError("[/pytorch/third_party/gloo/gloo/transport/tcp/pair.cc:547] Connection closed by peer "
                  "[127.0.0.1]:53398"), True),
    (RuntimeError("[../gloo/transport/tcp/unbound_buffer.cc:81] Timed out waiting 2000ms for recv operation "
                  "to complete"), True),
    # bugs whose text happens to contain the old substrings are NOT membership failures
    (RuntimeError("shape mismatch: peer tensor has 3 dims"), False),
    (RuntimeError("the operation timed out in user code"), False),
    (RuntimeError("socket option invalid in my config parser"), False),
    (XgmiError("xGMI all-reduce takes contiguous fp32 / bf16 tensors of 16-byte multiples"), False),
    (XgmiError("launch failed: hipError 98"), False),
    (dist.DistStoreError("store connection closed by peer"), False),   # the master itself: raise
    (ValueError("Connection closed by peer"), False),
    (TimeoutError("commit of step 4 timed out"), False),
])
def test_comm_error_classification_is_typed(exc, expect):
    assert is_comm_error(exc) is expect


class _DeadStoreRdzv:
    """A rendezvous client whose store stopped answering."""

    def aborted(self, epoch):
        raise dist.DistStoreError("Socket Timeout: recv() failed")


def test_watchdog_reports_a_dead_master_instead_of_swallowing_it(tmp_path, monkeypatch):
    monkeypatch.setenv("EDL_MASTER_TIMEOUT_S", "0.2")
    ctx = TrainerContext(job="wd", run_dir=str(tmp_path))
    tr = ElasticTrainer(lambda d: torch.nn.Linear(4, 4, device=d), device="cpu", ctx=ctx)
    tr.comm = LocalCommunicator(torch.device("cpu"))
    tr.rdzv = _DeadStoreRdzv()
    tr._start_watchdog()
    t_end = time.time() + 10
    while tr._master_lost is None and time.time() < t_end:
        time.sleep(0.02)
    tr._stop.set()
    assert tr._master_lost is not None and "DistStoreError" in tr._master_lost
    kinds = [r["kind"] for r in tr.events.records]
    assert kinds.count("store_unreachable") == 1 and "master_lost" in kinds
    assert tr.comm.aborted            # nothing may stay blocked in a collective
    assert issubclass(MasterUnreachable, RuntimeError) and not is_comm_error(MasterUnreachable("x"))
