"""Shipped MIOpen find-db for the ResNet-50 convolutions (NHWC bf16, gfx950, 256 CUs).

On its first call for a convolution shape, MIOpen benchmarks every applicable
solver (Find), including its naive reference kernels. For ResNet-50 at batch 256
on one MI355X that is 62 s before the first step (`profiles/r02_resnet50_miopen_db.txt`).
That delays every elastic joiner and every replacement worker by the same amount.
The search's winners are recorded in MIOpen's text find-db. With that file in
place, MIOpen goes straight to the recorded solver: 3.4 s to the first timed step on a fresh box.

MIOpen also writes to its user db, so :func:`install` copies the shipped file
into a per-user scratch directory and points ``MIOPEN_USER_DB_PATH`` there. It
does nothing when the user already set that variable, or when
``EDL_MIOPEN_DB=0``. It must run before the process's first convolution.
"""
from __future__ import annotations

import glob
import os
import shutil
import tempfile

SHIPPED_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tuned", "miopen")


def install(src_dir: str = SHIPPED_DIR) -> str | None:
    """Point MIOpen's user db at a scratch copy of the shipped find-db; returns that directory."""
    if os.environ.get("EDL_MIOPEN_DB", "1") == "0" or "MIOPEN_USER_DB_PATH" in os.environ:
        return None
    files = glob.glob(os.path.join(src_dir, "*.ufdb.txt"))
    if not files:
        return None
    dst = os.path.join(tempfile.gettempdir(), f"edl_miopen_db_{os.getuid()}")
    os.makedirs(dst, exist_ok=True)
    for f in files:
        out = os.path.join(dst, os.path.basename(f))
        if not os.path.exists(out):   # keep what MIOpen has added to an earlier copy
            shutil.copyfile(f, out)
    os.environ["MIOPEN_USER_DB_PATH"] = dst
    return dst
