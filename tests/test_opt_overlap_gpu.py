"""The optimizer update overlapping the next step's forward (ElasticTrainer._opt_overlap) gives
the same training as the serialized update, bit for bit.

The update runs on its own stream, group by group in the order the next forward reads them;
each module waits for its own parameters' update, each gradient write for the update that still
reads that gradient, and the transposed-weight cache refreshes each weight at its own first use.
A missing wait would let the forward read half-updated weights (or a backward overwrite gradients
the update has not read yet) and the two runs would drift apart."""
import pytest
import torch

from easydl_amd.models.llama import Llama, get_config
from easydl_amd.trainer.context import TrainerContext
from easydl_amd.trainer.data import SyntheticTokens
from easydl_amd.trainer.elastic import ElasticTrainer

pytestmark = pytest.mark.gpu
CFG = get_config("llama-tiny")


def _run(tmp, sub, cuda, overlap: bool, monkeypatch):
    from easydl_amd.ops import fused
    monkeypatch.setenv("EDL_OPT_OVERLAP", "1" if overlap else "0")
    monkeypatch.setattr(fused, "_WT_BATCH", fused._WT_BATCH)     # restored after the test
    ctx = TrainerContext(job="ovl", run_dir=str(tmp / sub))
    tr = ElasticTrainer(lambda d: Llama(CFG, device=d), global_batch=8, micro_batch=2, lr=1e-3, device=cuda,
                        ctx=ctx, seed=3)
    losses = []
    tr.fit(lambda m, b: m(*b), SyntheticTokens(CFG.vocab_size, 256, num_samples=4096), num_steps=8,
           on_step=lambda t, loss: losses.append(float(loss)))
    torch.cuda.synchronize()
    state = {f"data.{g.name}": g.data.clone() for g in tr.flat.groups}
    state.update({k: v.clone() for k, v in tr.opt.state_tensors().items()})
    return tr, losses, state


def test_overlapped_update_matches_the_serialized_one(cuda, tmp_path, monkeypatch):
    a, la, sa = _run(tmp_path, "serial", cuda, False, monkeypatch)
    assert a._opt_stream is None
    b, lb, sb = _run(tmp_path, "overlap", cuda, True, monkeypatch)
    assert b._opt_stream is not None
    assert la == lb
    for k in sa:
        assert torch.equal(sa[k], sb[k]), k
