"""Offline-tuned hipBLASLt / rocBLAS GEMM selections (PyTorch TunableOp).

hipBLASLt's heuristic picks a good kernel for most Llama shapes but not all
(the qkv projection forward gained 18 % from a tuned solution,
profiles/r01_gemm_shapes_hipblaslt.jsonl).  The framework ships the TunableOp
results for its own GEMM call forms on gfx950 (`easydl_amd/tuned/`), made by
one tuning run of the training step (``EDL_GEMM_TUNING=tune``); every later
run only reads the file (no tuning time, no GPU search).  GEMMs absent from
the file fall back to the library heuristic.

EDL_GEMM_TUNING: ``select`` (default: read the curated file, the
selections verified to speed up the whole step), ``use`` (read the full
round-1 file), ``tune`` (search every GEMM met and write the file at exit),
``off`` (library heuristics only).

Measured (profiles/r01_gemm_tuning_ab.jsonl): per GEMM the full set of tuned
selections is faster in TunableOp's isolated timing (lm_head 11.2 -> 8.5-9.1
ms, qkv 0.65 -> 0.53 ms), yet the full Llama-3-8B step ran 19,295 tokens/s
with them vs 19,496 without.  The curated file holds only the down-projection
weight gradient (dY^T [4096, M] @ h [M, 14336], M = 16384), the one GEMM the
heuristic runs at 1.13 PF/s: hipBLASLt solution 618613 takes it from 1.71 to
1.31 ms (scripts/gemm_wgrad_probe.py, profiles/r02_gemm_wgrad_probe.jsonl).
"""
from __future__ import annotations

import atexit
import logging
import os
import tempfile

log = logging.getLogger(__name__)
_TUNED_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tuned")
TUNED_FILE = os.path.join(_TUNED_DIR, "tunableop_gfx950.csv")
SELECT_FILE = os.path.join(_TUNED_DIR, "tunableop_gfx950_select.csv")


def apply(mode: str | None = None, path: str | None = None) -> str:
    """Configure TunableOp for this process; returns the mode in effect."""
    import torch
    mode = mode or os.environ.get("EDL_GEMM_TUNING", "select")
    path = path or os.environ.get("EDL_GEMM_TUNING_FILE") or (SELECT_FILE if mode == "select" else TUNED_FILE)
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
    # TunableOp READS the file named here when it starts (before read_file below) and writes it
    # at exit when it holds results that were not loaded: never the shipped file or the working
    # directory's default, and never a name another process writes -- an entry left there by
    # any earlier run would be taken as a selection (scripts/tunableop_scratch_probe.py: a
    # stale entry naming a solution this library lacks fails that GEMM).  With tuning off
    # nothing is written, so a per-process name does not pile up.
    tun.set_filename(os.path.join(tempfile.gettempdir(), f"edl_tunableop_scratch_{os.getuid()}_{os.getpid()}.csv"))
    ok = tun.read_file(path)
    if not ok:
        log.warning("TunableOp results %s not loaded (validator mismatch?): library heuristics", path)
        tun.enable(False)
        return "off"
    return mode
