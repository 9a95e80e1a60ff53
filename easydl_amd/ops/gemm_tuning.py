"""Offline-tuned hipBLASLt / rocBLAS GEMM selections (PyTorch TunableOp).

hipBLASLt's heuristic picks a good kernel for most Llama shapes but not all
(the qkv projection forward gained 18 % from a tuned solution,
profiles/r01_gemm_shapes_hipblaslt.jsonl).  The framework ships the TunableOp
results for its own GEMM call forms on gfx950 (`easydl_amd/tuned/`), made by
one tuning run of the training step (``EDL_GEMM_TUNING=tune``); every later
run only reads the file (no tuning time, no GPU search).  GEMMs absent from
the file fall back to the library heuristic.

EDL_GEMM_TUNING: ``off`` (default), ``use`` (read the shipped file),
``tune`` (search every GEMM met and write the file at exit).

Measured (profiles/r01_gemm_tuning_ab.jsonl): per GEMM the tuned selections
are faster in TunableOp's isolated timing (lm_head 11.2 -> 8.5-9.1 ms, qkv
0.65 -> 0.53 ms), yet the full Llama-3-8B step ran 19,295 tokens/s with them
vs 19,496 without — so the library heuristics stay the default.
"""
from __future__ import annotations

import atexit
import logging
import os

log = logging.getLogger(__name__)
TUNED_FILE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tuned",
                          "tunableop_gfx950.csv")


def apply(mode: str | None = None, path: str | None = None) -> str:
    """Configure TunableOp for this process; returns the mode in effect."""
    import torch
    mode = mode or os.environ.get("EDL_GEMM_TUNING", "off")
    path = path or TUNED_FILE
    if mode == "off" or not torch.cuda.is_available():
        return "off"
    import torch.cuda.tunable as tun
    if mode == "tune":
        tun.enable(True)
        tun.tuning_enable(True)
        tun.set_max_tuning_iterations(int(os.environ.get("EDL_GEMM_TUNING_ITERS", 10)))
        tun.set_max_tuning_duration(int(os.environ.get("EDL_GEMM_TUNING_MS", 10)))
        tun.set_filename(path)
        if hasattr(tun, "write_file"):
            atexit.register(tun.write_file)   # else TunableOp writes the file at process exit itself
        return "tune"
    if not os.path.exists(path):
        return "off"
    tun.enable(True)
    tun.tuning_enable(False)
    tun.set_filename(path)
    ok = tun.read_file(path)
    if not ok:
        log.warning("TunableOp results %s not loaded (validator mismatch?): library heuristics", path)
        tun.enable(False)
        return "off"
    return "use"
