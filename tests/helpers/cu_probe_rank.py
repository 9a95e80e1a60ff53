"""One training process for tests/test_brain_measured_gpu.py: a matrix-core-bound or an
HBM-bound model trained by ElasticTrainer (standalone) with the CU-sensitivity probe on; writes
the metrics record the rank would publish to the Brain (``_metrics_extra``) as JSON.

    python tests/helpers/cu_probe_rank.py compute|bandwidth OUT.json
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from easydl_amd.trainer.context import TrainerContext  # noqa: E402
from easydl_amd.trainer.elastic import ElasticTrainer  # noqa: E402


class GemvStack(torch.nn.Module):
    """Batch-1 matrix-vector layers: every forward/backward kernel streams a 128 MB weight (or
    its gradient) through HBM once per step -- bandwidth-bound, whatever the code calls it."""

    def __init__(self, width=8192, layers=6, device=None):
        super().__init__()
        self.layers = torch.nn.ModuleList(torch.nn.Linear(width, width, bias=False, device=device,
                                                          dtype=torch.bfloat16) for _ in range(layers))

    def forward(self, x):
        for lin in self.layers:
            x = torch.tanh(lin(x))
        return x.float().square().mean()


class Vectors:
    def __init__(self, width):
        self.width = width

    def __len__(self):
        return 1 << 16

    def batch(self, idx, device):
        g = torch.Generator().manual_seed(int(list(idx)[0]))
        return torch.randn(len(list(idx)), self.width, generator=g).to(device, torch.bfloat16)


def main(kind: str, out: str) -> None:
    os.environ.setdefault("EDL_CU_PROBE_EVERY", "4")
    dev = torch.device("cuda", 0)
    ctx = TrainerContext(job=f"cu-{kind}", run_dir=os.path.join(os.path.dirname(out), kind))
    if kind == "compute":
        from easydl_amd.models.llama import Llama, get_config
        from easydl_amd.trainer.data import SyntheticTokens
        cfg = get_config("llama-tiny", dim=2048, n_layers=4, n_heads=16, n_kv_heads=4, ffn_dim=8192,
                         vocab_size=8192, max_seq_len=2048)
        tr = ElasticTrainer(lambda d: Llama(cfg, device=d), global_batch=8, micro_batch=4, device=dev, ctx=ctx)
        tr.fit(lambda m, b: m(*b), SyntheticTokens(cfg.vocab_size, 2048, num_samples=4096), num_steps=24)
    else:
        tr = ElasticTrainer(lambda d: GemvStack(device=d), global_batch=2, micro_batch=1, device=dev, ctx=ctx)
        tr.fit(lambda m, x: m(x), Vectors(8192), num_steps=60)
    torch.cuda.synchronize(dev)
    rec = tr._metrics_extra()
    tr.close()
    with open(out, "w") as f:
        json.dump(rec, f)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
