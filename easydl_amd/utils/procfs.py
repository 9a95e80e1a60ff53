"""Process state from /proc (no torch import: the operator uses it)."""
from __future__ import annotations

import os


def mm_released(pid: int) -> bool:
    """True once no thread of ``pid`` holds its address space any more, or it is gone.

    A SIGKILLed process first detaches its address space from every thread; the last
    thread to do so tears it down, and that teardown starts by releasing the process's
    GPU context (the amdkfd MMU notifier destroys its queues) before the long part, the
    page tables.  From here on the process runs no more GPU work."""
    try:
        tids = os.listdir(f"/proc/{pid}/task")
    except OSError:
        return True
    for tid in tids:
        try:
            with open(f"/proc/{pid}/task/{tid}/status") as f:
                if "VmRSS:" in f.read():
                    return False
        except OSError:
            continue
    return True


def exit_status(pid: int) -> int | None:
    """The wait status a dying (or zombie) process will report (/proc/<pid>/stat field 52,
    set at the start of its exit), or None if it is gone or the field is unavailable.
    0: a normal exit(0); a SIGKILL reads 9."""
    try:
        with open(f"/proc/{pid}/stat") as f:
            fields = f.read().rsplit(")", 1)[1].split()
        return int(fields[49])       # field 52; fields[0] is field 3 (state)
    except (OSError, IndexError, ValueError):
        return None
