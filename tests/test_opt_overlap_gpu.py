"""The optimizer update overlapping the next step's forward (ElasticTrainer._opt_overlap) gives
the same training as the serialized update, bit for bit.

The update runs on its own stream, group by group in the order the next forward reads them;
each module waits for its own parameters' update, each gradient write for the update that still
reads that gradient, the transposed-weight cache refreshes each weight at its own first use, and
the update itself waits for the step's backward (ElasticTrainer._order_update_after_step).
A missing wait would let the forward read half-updated weights (or the update read gradients
the backward has not written yet) and the two runs would drift apart.

llama-tiny is host-bound: left alone, each backward finishes on the GPU before the host queues
the update, and no missing edge could show.  So every micro-batch starts with a GPU spin
(``torch.cuda._sleep``) that keeps the compute stream well behind the host, and the losses stay
on the GPU until the run ends (no per-step ``float(loss)`` sync).  The negative control removes
the per-step update->backward edge at the stream level and must see the update run ahead."""
import pytest
import torch

from easydl_amd.models.llama import Llama, get_config
from easydl_amd.trainer.context import TrainerContext
from easydl_amd.trainer.data import SyntheticTokens
from easydl_amd.trainer.elastic import ElasticTrainer

pytestmark = pytest.mark.gpu
CFG = get_config("llama-tiny")
# ~50 ms of spinning per micro-batch: the GPU lags the host by steps however slow the host is (at
# ~10 ms the full GPU tier once saw the host's own per-step time cover the lag: no race to expose)
LAG_CYCLES = 100_000_000


def _run(tmp, sub, cuda, overlap: bool, monkeypatch):
    from easydl_amd.ops import fused
    monkeypatch.setenv("EDL_OPT_OVERLAP", "1" if overlap else "0")
    monkeypatch.setattr(fused, "_WT_BATCH", fused._WT_BATCH)     # restored after the test
    ctx = TrainerContext(job="ovl", run_dir=str(tmp / sub))
    tr = ElasticTrainer(lambda d: Llama(CFG, device=d), global_batch=8, micro_batch=2, lr=1e-3, device=cuda,
                        ctx=ctx, seed=3)
    losses = []

    def loss_fn(m, b):
        torch.cuda._sleep(LAG_CYCLES)     # the compute stream falls behind the host here
        return m(*b)
    tr.fit(loss_fn, SyntheticTokens(CFG.vocab_size, 256, num_samples=4096), num_steps=8,
           on_step=lambda t, loss: losses.append(loss.detach().clone()))
    torch.cuda.synchronize()
    state = {f"data.{g.name}": g.data.clone() for g in tr.flat.groups}
    state.update({k: v.clone() for k, v in tr.opt.state_tensors().items()})
    return tr, [float(x) for x in losses], state


def test_overlapped_update_matches_the_serialized_one(cuda, tmp_path, monkeypatch):
    a, la, sa = _run(tmp_path, "serial", cuda, False, monkeypatch)
    assert a._opt_stream is None
    b, lb, sb = _run(tmp_path, "overlap", cuda, True, monkeypatch)
    assert b._opt_stream is not None
    assert la == lb
    for k in sa:
        assert torch.equal(sa[k], sb[k]), k


def test_update_stream_waits_for_the_step_only_through_the_edge(cuda, tmp_path, monkeypatch):
    """Negative control at the stream level (deterministic, unlike a race): with the compute
    stream busy for ~200 ms, work queued on the update stream after ``_order_update_after_step``
    waits for it; without that edge it runs at once -- the update would read gradients the
    backward has not written.  (An end-to-end racy run showed the divergence when run alone, but
    inside the full GPU tier the race did not always land; the edge itself is what must hold.)"""
    import time
    tr, _, _ = _run(tmp_path, "edge", cuda, True, monkeypatch)
    ovl = tr._opt_stream
    assert ovl is not None
    cur = torch.cuda.current_stream(cuda)
    torch.cuda.synchronize()

    def queued_after(edge: bool) -> bool:
        torch.cuda._sleep(LAG_CYCLES * 4)             # ~200 ms on the compute stream
        if edge:
            tr._order_update_after_step(ovl)
        ev = torch.cuda.Event()
        ev.record(ovl)
        t_end = time.perf_counter() + 0.05
        done = False
        while time.perf_counter() < t_end and not done:
            done = ev.query()
        still_busy = not cur.query()
        torch.cuda.synchronize()
        assert still_busy, "the compute stream finished its spin too early for the check"
        return not done

    assert queued_after(True), "the update stream ran ahead of the step despite the edge"
    assert not queued_after(False), "without the edge the update stream should not wait"
