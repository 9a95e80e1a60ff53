"""Llama training entry point for `edl submit` (all-reduce mode, in-memory snapshots).

Env: EDL_MODEL (llama3-8b), EDL_SEQ, EDL_MBS, EDL_ACCUM, EDL_STEPS, EDL_CKPT_INTERVAL,
EDL_PLANNED_WORKERS (global batch = planned workers x MBS x ACCUM, kept across resizes).
"""
import os

import torch

from easydl_amd.ckpt.manager import CheckpointManager
from easydl_amd.models.llama import Llama, get_config
from easydl_amd.trainer.data import SyntheticTokens
from easydl_amd.trainer.elastic import ElasticTrainer


def main():
    e = os.environ
    cfg = get_config(e.get("EDL_MODEL", "llama3-8b"))
    seq, mbs, accum = int(e.get("EDL_SEQ", 8192)), int(e.get("EDL_MBS", 1)), int(e.get("EDL_ACCUM", 1))
    world = int(e.get("EDL_PLANNED_WORKERS", torch.cuda.device_count() or 1))
    ckpt = CheckpointManager(e.get("EDL_JOB", "llama"), interval=int(e.get("EDL_CKPT_INTERVAL", 50)))
    tr = ElasticTrainer(lambda d: Llama(cfg, device=d), global_batch=world * mbs * accum, micro_batch=mbs,
                        checkpoint=ckpt, log_every=10)
    tr.tokens_per_sample = seq
    tr.fit(lambda m, b: m(*b), SyntheticTokens(cfg.vocab_size, seq), num_steps=int(e.get("EDL_STEPS", 100)))
    tr.close()
    ckpt.close()


if __name__ == "__main__":
    main()
