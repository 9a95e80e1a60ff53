"""roctx ranges for rocprofv3 ``--marker-trace``.

``with trace.range("bwd"):`` pushes/pops a roctx range through the native
runtime (dlopen'ed profiler SDK); disabled unless ``EDL_TRACE=1`` so the hot
loop pays nothing by default.
"""
from __future__ import annotations

import contextlib
import os

_enabled = os.environ.get("EDL_TRACE", "0") == "1"
_rt = None


def enabled() -> bool:
    return _enabled


def enable(on: bool = True) -> None:
    global _enabled
    _enabled = on


def _runtime():
    global _rt
    if _rt is None:
        from easydl_amd import _native
        _rt = _native.runtime() if _native.runtime_available() else False
    return _rt


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors roctx naming
    rt = _runtime() if _enabled else None
    if rt:
        rt("edl_roctx_push", name.encode())
    try:
        yield
    finally:
        if rt:
            rt("edl_roctx_pop")


def mark(name: str) -> None:
    rt = _runtime() if _enabled else None
    if rt:
        rt("edl_roctx_mark", name.encode())
