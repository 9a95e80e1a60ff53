"""Tensor parallel Llama (TP=2 over gloo) == dense model: loss and every sharded grad."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("sp,overlap", [("0", "0"), ("0", "1"), ("1", "0")])
def test_tp2_matches_dense(tmp_path, sp, overlap):
    """sp=1: Megatron sequence parallelism (token-sharded residual stream and norms);
    overlap=1: row-parallel outputs all-reduced chunk by chunk (8-row chunks here) and
    column-parallel input gradients all-reduced under the weight-gradient GEMMs."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = [subprocess.Popen([sys.executable, os.path.join(ROOT, "tests/helpers/tp_worker.py")],
                              env=dict(os.environ, RANK=str(r), WORLD_SIZE="2", PORT=str(port),
                                       OUT=str(tmp_path / "r"), PYTHONPATH=ROOT, SP=sp, EDL_TP_OVERLAP=overlap,
                                       EDL_TP_CHUNK_ROWS="8")) for r in range(2)]
    assert [p.wait(timeout=120) for p in procs] == [0, 0]
    for r in range(2):
        res = json.load(open(tmp_path / f"r.{r}"))
        assert abs(res["loss_d"] - res["loss_t"]) < 1e-5, res
        assert res["grad_rel_err"] < 1e-4, res
        # 2 layers x (2 row-parallel outputs in 4 chunks + 2 column-parallel dX) + LM-head dX
        assert res["async_starts"] == (2 * (2 * 4 + 2) + 1 if overlap == "1" else 0), res


class _ThreadGroup:
    """TP group of `size` threads in ONE process (one GPU): all_reduce / all_reduce_max
    meet at a barrier and combine every thread's tensor."""

    def __init__(self, size, rank, shared):
        self.size, self.rank, self.shared = size, rank, shared

    def _combine(self, x, op):
        import threading  # noqa: F401
        sh = self.shared
        sh["bufs"][self.rank] = x
        sh["barrier"].wait()
        out = sh["bufs"][0].clone()
        for t in sh["bufs"][1:]:
            out = torch.maximum(out, t) if op == "max" else out + t
        sh["barrier"].wait()
        return out

    def all_reduce(self, x):
        return self._combine(x.contiguous(), "sum")

    def all_reduce_max(self, x):
        return self._combine(x.contiguous(), "max")


@pytest.mark.gpu
@pytest.mark.parametrize("tp", [2, 4])
def test_vocab_parallel_xent_kernel_matches_dense(cuda, tp):
    """edl_xent_vp + (MAX, SUM) exchange == the dense fp32 cross entropy: loss and the
    in-place logits gradient of every vocab shard (incl. ignored rows)."""
    import threading

    import torch.nn.functional as F

    from easydl_amd.parallel.tp import vocab_parallel_cross_entropy
    torch.manual_seed(0)
    T, V = 96, 1024
    full = (torch.randn(T, V, device=cuda) * 3).to(torch.bfloat16)
    labels = torch.randint(0, V, (T,), device=cuda)
    labels[::7] = -100
    ref_in = full.float().requires_grad_()
    ref = F.cross_entropy(ref_in, labels, ignore_index=-100)
    ref.backward()
    shared = {"bufs": [None] * tp, "barrier": threading.Barrier(tp)}
    out, grads = [None] * tp, [None] * tp
    vs = V // tp

    def rank(r):
        torch.cuda.set_device(cuda)
        x = full[:, r * vs:(r + 1) * vs].clone().requires_grad_()
        loss = vocab_parallel_cross_entropy(x, labels, r * vs, _ThreadGroup(tp, r, shared))
        loss.backward()
        out[r], grads[r] = loss.detach(), x.grad

    ts = [threading.Thread(target=rank, args=(r,)) for r in range(tp)]
    [t.start() for t in ts]
    [t.join(60) for t in ts]
    torch.cuda.synchronize()
    for r in range(tp):
        assert abs(out[r].item() - ref.item()) < 1e-3 * max(1.0, abs(ref.item())), (out[r].item(), ref.item())
        g = grads[r].float()
        gr = ref_in.grad[:, r * vs:(r + 1) * vs]
        assert (g - gr).abs().max().item() < 2e-3, (g - gr).abs().max().item()


def test_tp_shard_dry_run_on_cpu(tmp_path):
    """trainer/tp_dryrun.py (config-5 sizing): one TP shard at full depth against a loopback
    TP group -- here a tiny Llama on the CPU, with and without recompute: real steps, the
    TP collective bytes a real group would move, and the snapshot-mode decision."""
    from easydl_amd.trainer import tp_dryrun
    for rc in (True, False):
        r = tp_dryrun.run("llama-tiny", 2, 1, 32, 2, 2, 2, 1, rc, device="cpu")
        assert r["recompute"] == rc and r["layers"] == 2 and r["ms_per_step"] > 0
        assert r["tp_collective_bytes_per_step_per_rank"] > 0
        snap = r["snapshot"]
        assert snap["mode"] in ("full", "lean", "off") and snap["full_bytes"] > snap["lean_bytes"]
        assert r["loss"] == r["loss"]
