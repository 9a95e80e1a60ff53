"""One rank of tests/test_grad_parity_cpu.py (launched by torch.distributed.run): llama-tiny trained
by ElasticTrainer for EDL_PARITY_STEPS steps with bf16 or fp32 gradient buffers (the bucketed
all-reduce runs in that dtype over gloo); rank 0 saves the initial and final flat weights."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from easydl_amd.models.llama import Llama, get_config  # noqa: E402
from easydl_amd.trainer.data import SyntheticTokens  # noqa: E402
from easydl_amd.trainer.elastic import ElasticTrainer  # noqa: E402


def main(grad: str, out: str) -> None:
    torch.set_num_threads(1)
    cfg = get_config("llama-tiny")
    gd = torch.bfloat16 if grad == "bf16" else torch.float32
    tr = ElasticTrainer(lambda d: Llama(cfg, device=d, dtype=torch.float32), global_batch=16, micro_batch=1,
                        lr=2e-3, device="cpu", grad_dtype=gd, seed=11)
    init = torch.cat([g.data.detach().clone().view(-1) for g in tr.flat.groups])
    losses = []
    tr.fit(lambda m, b: m(*b), SyntheticTokens(cfg.vocab_size, 64, num_samples=4096),
           num_steps=int(os.environ.get("EDL_PARITY_STEPS", 50)), on_step=lambda t, l: losses.append(float(l)))
    final = torch.cat([g.data.detach().clone().view(-1) for g in tr.flat.groups])
    if tr.comm.rank == 0:
        torch.save({"init": init, "final": final, "losses": losses, "world": tr.comm.world_size,
                    "grad_dtype": str(tr.flat.grad_dtype)}, out)
    tr.close()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
