"""HIP graph replay of a fixed-shape forward (utils/graphs.py): BERT-large inference at batch 1
x 128 tokens -- ~300 kernels of a few microseconds, each paying a host launch when eager -- as
one graph launch.  Same kernels, same order: the logits are bit-identical to eager."""
import time

import pytest
import torch

from easydl_amd.utils.graphs import GraphedCallable


def test_graphed_callable_rejects_host_tensors():
    with pytest.raises(TypeError):
        GraphedCallable(lambda x: x)(torch.zeros(2))


def _timed(fn, x, iters=30):
    fn(x)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn(x)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


@pytest.mark.gpu
def test_graphed_bert_forward_is_exact_faster_and_sees_new_weights(cuda):
    from easydl_amd.models.bert import BERT_LARGE, BertMLM
    torch.manual_seed(0)
    m = BertMLM(BERT_LARGE, device=cuda).eval()
    fwd = lambda ids: m(ids)  # noqa: E731
    g = GraphedCallable(fwd)
    ids = torch.randint(0, BERT_LARGE.vocab_size, (1, 128), device=cuda)
    with torch.no_grad():
        ref = fwd(ids)
    out = g(ids)
    assert torch.equal(out, ref)
    # another batch of the same shape: the captured buffers take the new input
    ids2 = torch.randint(0, BERT_LARGE.vocab_size, (1, 128), device=cuda)
    with torch.no_grad():
        ref2 = fwd(ids2)
    assert torch.equal(g(ids2), ref2) and g.captures == 1
    with torch.no_grad():
        t_eager = min(_timed(fwd, ids) for _ in range(2))
    t_graph = min(_timed(g, ids) for _ in range(2))
    print(f"\n[hip-graph] bert-large fwd 1x128: eager {t_eager * 1e3:.3f} ms, graph {t_graph * 1e3:.3f} ms, "
          f"{t_eager / t_graph:.2f}x")
    assert t_graph < t_eager / 1.2, (t_eager, t_graph)
    # weights are read in place: an update (a new snapshot loaded by the evaluator) is seen
    with torch.no_grad():
        m.head_w.mul_(0.5)
        ref3 = fwd(ids)
    assert torch.equal(g(ids).clone(), ref3) and not torch.equal(ref3, ref)
    # a new shape is a new capture
    ids4 = torch.randint(0, BERT_LARGE.vocab_size, (2, 64), device=cuda)
    with torch.no_grad():
        ref4 = fwd(ids4)
    assert torch.equal(g(ids4), ref4) and g.captures == 2


def test_graphed_wrapper_is_the_module_on_the_cpu():
    from easydl_amd.utils.graphs import graphed
    m = torch.nn.Linear(4, 4)
    assert graphed(m) is m


@pytest.mark.gpu
def test_graphed_module_delegates_attributes_and_calls(cuda):
    from easydl_amd.utils.graphs import GraphedModule, graphed
    m = torch.nn.Sequential(torch.nn.Linear(64, 64), torch.nn.ReLU(), torch.nn.Linear(64, 8)).to(cuda)
    g = graphed(m)
    assert isinstance(g, GraphedModule) and g.training == m.training
    assert [p.data_ptr() for p in g.parameters()] == [p.data_ptr() for p in m.parameters()]
    x = torch.randn(16, 64, device=cuda)
    with torch.no_grad():
        assert torch.equal(g(x), m(x))


@pytest.mark.gpu
def test_a_forward_that_syncs_with_the_host_falls_back_to_eager(cuda):
    def fn(x):
        n = int((x > 0).sum())            # host sync: not capturable
        return x * n
    g = GraphedCallable(fn)
    x = torch.randn(32, device=cuda)
    assert torch.equal(g(x), fn(x)) and g.captures == 0
    assert torch.equal(g(x), fn(x))


@pytest.mark.gpu
def test_snapshot_evaluator_scores_through_hip_graphs(cuda, tmp_path):
    """The evaluator's model calls replay graphs by default; the loss equals the eager one."""
    from easydl_amd.ckpt.manager import CheckpointManager, unlink_job_segments
    from easydl_amd.models.llama import Llama, get_config
    from easydl_amd.trainer.context import TrainerContext
    from easydl_amd.trainer.data import SyntheticTokens
    from easydl_amd.trainer.elastic import ElasticTrainer
    from easydl_amd.trainer.evaluator import SnapshotEvaluator
    cfg = get_config("llama-tiny")
    unlink_job_segments("gev")
    data = SyntheticTokens(cfg.vocab_size, 128, num_samples=1024)
    ckpt = CheckpointManager("gev", interval=2)
    try:
        tr = ElasticTrainer(lambda d: Llama(cfg, device=d), global_batch=4, micro_batch=2, lr=1e-3, device=cuda,
                            ctx=TrainerContext(job="gev", run_dir=str(tmp_path)), checkpoint=ckpt)
        tr.fit(lambda m, b: m(*b), data, num_steps=4)
        torch.cuda.synchronize()
        batch = list(data.batch([1, 2, 3, 4], cuda))
        res = {}
        for g in (False, True):
            ev = SnapshotEvaluator(lambda d: Llama(cfg, device=d), "gev", device=cuda, run_dir=str(tmp_path))
            seen = []
            res[g] = ev.run(lambda m: (seen.append(type(m).__name__), {"loss": float(m(*batch))})[1],
                            interval_s=0, max_evals=1, graphed=g)
            assert seen == (["GraphedModule"] if g else ["Llama"])
        assert res[True][0]["step"] == res[False][0]["step"] == 4
        assert res[True][0]["loss"] == res[False][0]["loss"]
        tr.close()
    finally:
        unlink_job_segments("gev")
