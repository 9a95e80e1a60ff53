"""Worker script for multi-process elastic tests (CPU/gloo).

Env: EDL_* contract (or torchrun-style RANK/WORLD_SIZE/MASTER_*), plus
TEST_STEPS, TEST_GB (global batch), TEST_OUT (result json path).
"""
import hashlib
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from easydl_amd.models.llama import Llama, get_config  # noqa: E402
from easydl_amd.trainer.data import SyntheticTokens  # noqa: E402
from easydl_amd.trainer.elastic import ElasticTrainer  # noqa: E402

torch.set_num_threads(1)
cfg = get_config("llama-tiny", n_layers=1, dim=64, n_heads=4, n_kv_heads=2, ffn_dim=128, vocab_size=128)
steps = int(os.environ.get("TEST_STEPS", 8))
gb = int(os.environ.get("TEST_GB", 6))
if int(os.environ.get("EDL_TP", 1)) > 1:
    from easydl_amd.parallel.tp import LlamaTP  # noqa: E402
    model_fn = lambda dev, g: LlamaTP(cfg, g, device=dev, dtype=torch.float32)  # noqa: E731
else:
    model_fn = lambda dev: Llama(cfg, device=dev, dtype=torch.float32)  # noqa: E731
ckpt = None
if os.environ.get("TEST_CKPT"):
    from easydl_amd.ckpt.manager import CheckpointManager  # noqa: E402
    ckpt = CheckpointManager(os.environ["TEST_CKPT_JOB"], interval=int(os.environ["TEST_CKPT"]), pin=False)
tr = ElasticTrainer(model_fn, global_batch=gb, micro_batch=2, lr=1e-3, device="cpu", checkpoint=ckpt,
                    moment_dtype=os.environ.get("TEST_MOMENTS", "fp32"))
tr.fit(lambda m, b: m(*b), SyntheticTokens(cfg.vocab_size, 16, num_samples=4096), num_steps=steps,
       on_step=lambda t, l: time.sleep(float(os.environ.get("TEST_STEP_SLEEP", 0))))
h = hashlib.sha256()
for g in (tr.flat.groups if tr.flat is not None else []):
    h.update(g.data.numpy().tobytes())
hs = hashlib.sha256(h.digest())
for t in (tr.opt.state_tensors().values() if tr.opt is not None else []):
    hs.update(t.contiguous().view(torch.uint8).numpy().tobytes())     # master AND moments
res = {"index": tr.ctx.index, "step": tr.step, "hash": h.hexdigest(), "tp_rank": tr.held_tp,
       "state_hash": hs.hexdigest(), "snapshot_mode": getattr(ckpt, "mode", None),
       "moment_dtype": str(getattr(tr.opt, "moment_dtype", "")).replace("torch.", ""),
       "dp_rank": tr.dp_comm.rank if tr.dp_comm is not None else None,
       "worlds": [r["world"] for r in tr.history], "epochs": [r["epoch"] for r in tr.history],
       "loss": float(tr.last_loss) if tr.last_loss is not None else None,
       "bucket_mb": tr.ddp.bucket_mb if tr.ddp is not None else None, "plan_version": tr.plan_version}
out = os.environ.get("TEST_OUT") or os.path.join(os.environ["EDL_RUN_DIR"], f"res{tr.ctx.index}-{os.getpid()}.json")
with open(out, "w") as f:
    json.dump(res, f)
tr.close()
if ckpt is not None:
    ckpt.close()
