"""``moment_dtype="auto"`` is one decision per job: the first process publishes its pick
in the job store and every later one adopts it; a replacement that adopts a dead worker's HBM keeps
that worker's moment dtype; and a snapshot whose tensors have another dtype than the restoring
process's buffers is refused loudly instead of being copied as raw bytes."""
import numpy as np
import pytest
import torch
import torch.distributed as dist

from easydl_amd.ckpt.manager import _load_shard
from easydl_amd.master.store import KV
from easydl_amd.models.llama import Llama, get_config
from easydl_amd.trainer.context import TrainerContext
from easydl_amd.trainer.elastic import ElasticTrainer
from easydl_amd.utils import vram

CFG = get_config("llama-tiny", n_layers=1, dim=64, n_heads=4, n_kv_heads=2, ffn_dim=128, vocab_size=128)


class _Budget:
    """Checkpoint stand-in whose host budget fits two bf16-moment slots but not two fp32 ones."""
    stats: dict = {}

    def __init__(self, pick_bf16: bool):
        self.pick_bf16 = pick_bf16

    def host_budget_bytes(self, tr):
        n = sum(g.numel for g in tr.flat.groups)
        return 2 * n * 10 if self.pick_bf16 else 2 * n * 20


def _trainer(tmp_path, pick_bf16: bool) -> ElasticTrainer:
    ctx = TrainerContext(job="md", run_dir=str(tmp_path))
    return ElasticTrainer(lambda d: Llama(CFG, device=d), device="cpu", ctx=ctx, moment_dtype="auto",
                          checkpoint=_Budget(pick_bf16))


def test_first_pick_is_published_and_later_processes_adopt_it(tmp_path):
    kv = KV(dist.HashStore(), "edl/md")
    a = _trainer(tmp_path / "a", pick_bf16=True)
    assert a.opt.moment_dtype == torch.bfloat16
    a.kv = kv
    a._agree_moment_dtype()
    assert kv.get_str("job/moment_dtype") == "bf16"
    # a process whose own host budget says fp32 (e.g. the dead worker's segments still fill /dev/shm)
    b = _trainer(tmp_path / "b", pick_bf16=False)
    assert b.opt.moment_dtype == torch.float32
    b.kv = kv
    b._agree_moment_dtype()
    assert b.opt.moment_dtype == torch.bfloat16
    assert all(st["m"].dtype == torch.bfloat16 and st["v"].dtype == torch.bfloat16 for st in b.opt.state)
    assert kv.get_str("job/moment_dtype") == "bf16"
    # a process built after the decision reads it before choosing
    c = _trainer(tmp_path / "c", pick_bf16=False)
    c.kv = kv
    assert c._choose_moment_dtype("auto") == torch.bfloat16


def test_takeover_keeps_the_adopted_moment_dtype(tmp_path):
    vram.adopt({"opt/decay0/m": torch.zeros(4, dtype=torch.bfloat16)})
    try:
        tr = _trainer(tmp_path, pick_bf16=False)     # its own budget would say fp32
        assert tr.opt.moment_dtype == torch.bfloat16
    finally:
        vram.release_unused()
        vram.TAKEN.clear()
        vram.ADOPTED_FROM.clear()


def test_restore_refuses_a_snapshot_of_another_dtype():
    dst = {"opt.g.m": torch.zeros(8, dtype=torch.float32)}
    raw = np.zeros(64, dtype=np.uint8)
    table = [["opt.g.m", "bfloat16", 8, 0, 8, 0]]
    with pytest.raises(RuntimeError, match="refusing to restore"):
        _load_shard(lambda off, nb: raw[off:off + nb], table, dst, torch.device("cpu"), 0, "test shard")
