"""Mid-step resume from the HOST gradient shadow (utils/gshadow.py) on the GPU.

The worker copies its accumulated gradients device -> host after each micro-batch, group by
group, while the next micro-batch runs; each parameter's next gradient write waits only for its
group's copy (gradsink.await_shadow).  It dies before micro-batch 2 of step 4 (its gradient
buffers torn by an in-flight backward); the replacement adopts its HBM (weights, master, moments),
loads the host shadow (micro-batches 0-1) and runs micro-batches 2-3: the result is bit-identical
to an uninterrupted run.  A missing wait would let a write race the copy and tear the shadow."""
import os
import subprocess

import pytest
import torch

from easydl_amd.ckpt.manager import CheckpointManager, unlink_job_segments
from easydl_amd.models.llama import Llama, get_config
from easydl_amd.trainer.context import TrainerContext
from easydl_amd.trainer.data import SyntheticTokens
from easydl_amd.trainer.elastic import ElasticTrainer
from easydl_amd.utils import stepmarks, vram
from easydl_amd.utils.gshadow import HostShadow

pytestmark = pytest.mark.gpu
CFG = get_config("llama-tiny")
JOB = "hshadow"


def _mk(tmp, sub, seed, dev, ckpt=None):
    ctx = TrainerContext(job=JOB, run_dir=str(tmp / sub))
    return ElasticTrainer(lambda d: Llama(CFG, device=d), global_batch=8, micro_batch=2, lr=1e-3, device=dev,
                          ctx=ctx, checkpoint=ckpt, seed=seed)


def _state(t):
    out = {f"data.{g.name}": g.data.clone() for g in t.flat.groups}
    out.update({k: v.clone() for k, v in t.opt.state_tensors().items()})
    return out


def test_mid_step_resume_from_the_host_shadow_is_bit_exact(cuda, tmp_path, monkeypatch):
    unlink_job_segments(JOB)
    data = SyntheticTokens(CFG.vocab_size, 128, num_samples=4096)
    p = subprocess.Popen(["true"])
    p.wait()
    dead = p.pid
    a = _mk(tmp_path, "dead", 1, cuda)
    a.fit(lambda m, b: m(*b), data, num_steps=3)
    slot = f"{a.ctx.role}{a.ctx.index}"
    a._marks = stepmarks.StepMarks(JOB, slot, device=cuda)          # GPU-written marks
    hs = HostShadow(JOB, slot, a.flat.groups)
    a._hshadow, a._hshadow_views = hs, [(hs.group_views(i), hs.loss_view(i)) for i in (0, 1)]
    calls = {"n": 0}

    def dies(m, b):
        calls["n"] += 1
        if calls["n"] == 3:
            raise KeyboardInterrupt("killed before micro-batch 2 of step 4")
        return m(*b)
    try:
        a.fit(dies, data, num_steps=4)
    except KeyboardInterrupt:
        pass
    torch.cuda.synchronize()
    # two slots, alternating: micro-batch 0's sum in slot 0, micro-batches 0-1 in slot 1
    assert a.step == 3 and (a._marks.read_shadow(0), a._marks.read_shadow(1)) == ((4, 1), (4, 2))
    for g in a.flat.groups:
        g.grad.add_(1.0)            # the in-flight backward's partial adds: the shadow must be used
    exported = {k: t.clone() for k, t in a.vram_state_tensors().items()}
    assert not any("gshadow" in k for k in exported)        # host shadow: nothing extra in HBM
    hs.close()
    a._marks.close()
    monkeypatch.setattr(stepmarks, "read_slot",
                        lambda job, s, shadow=False: (3, 3, dead) + ((4, 1, 4, 2) if shadow else ()))
    vram.adopt(exported, pid=dead)
    ck = CheckpointManager(JOB, interval=100)
    try:
        b = _mk(tmp_path, "b", 5, cuda, ck)
        b.fit(lambda m, x: m(*x), data, num_steps=6)
        ev = [r for r in b.events.records if r["kind"] in ("restored", "resumed_mid_step", "grad_shadow_loaded")]
        kinds = [r["kind"] for r in ev]
        assert kinds == ["restored", "grad_shadow_loaded", "resumed_mid_step"], ev
        assert ev[2]["micro_batches_done"] == 2 and ev[2]["host"] is True and ev[1]["slot"] == 1
        vram.adopt({})
        ref = _mk(tmp_path, "ref", 1, cuda).fit(lambda m, x: m(*x), data, num_steps=6)
        got, want = _state(b), _state(ref)
        for k in want:
            assert torch.equal(got[k], want[k]), k
    finally:
        ck.close()
        vram.adopt({})
        unlink_job_segments(JOB)
        assert not os.path.exists(f"/dev/shm/edl-{JOB}-gshadow-{slot}")
