"""Can a side thread grow the caching allocator (fresh HBM: slow to hand out) while the main
thread keeps launching work from blocks it already holds?  If the allocator's lock is held
across hipMalloc, the main thread stalls for the whole growth.

    python scripts/bg_grow_probe.py            # calm GPU: one JSON line
    python scripts/bg_grow_probe.py after-kill # right after a process holding 180 GB was SIGKILLed
                                               # (scripts/realloc_probe.py's victim): growth alone,
                                               # then growth in a thread under a main loop
"""
import json
import os
import signal
import subprocess
import sys
import threading
import time

import torch


def _kill_victim():
    here = os.path.dirname(os.path.abspath(__file__))
    v = subprocess.Popen([sys.executable, os.path.join(here, "realloc_probe.py"), "victim"],
                         stdout=subprocess.PIPE, text=True)
    assert v.stdout.readline().strip() == "ready"
    time.sleep(1.0)
    v.send_signal(signal.SIGKILL)
    v.wait()


def main(after_kill=False, threaded=True):
    dev = torch.device("cuda", 0)
    a = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    blk = torch.empty(256 << 20, dtype=torch.uint8, device=dev)
    del blk                                           # one cached 256 MB block for the main loop
    torch.cuda.synchronize()
    if after_kill:
        _kill_victim()
    t0 = time.perf_counter()
    if not threaded:
        x = torch.empty(int(48e9), dtype=torch.uint8, device=dev)
        print(json.dumps({"after_kill": after_kill, "grow48g_alone_s": round(time.perf_counter() - t0, 3)}),
              flush=True)
        return
    out = {"after_kill": after_kill}
    done = {}

    def grow():
        t = time.perf_counter()
        y = torch.empty(int(48e9), dtype=torch.uint8, device=dev)
        done["grow_s"] = time.perf_counter() - t
        done["end"] = time.perf_counter()
        del y

    iters = []
    th = None
    for i in range(400):
        t = time.perf_counter()
        b = torch.empty(256 << 20, dtype=torch.uint8, device=dev)   # from the cache
        a = torch.mm(a, a)
        a = a / 64.0
        del b
        if i % 8 == 0:
            torch.cuda.synchronize()
        iters.append((t, time.perf_counter() - t))
        if i == 40:
            th = threading.Thread(target=grow)
            th.start()
            start = time.perf_counter()
    th.join()
    during = [d for t, d in iters if start <= t <= done["end"]]
    before = sorted(d for t, d in iters[:40])
    out.update(grow48g_in_thread_s=round(done["grow_s"], 3), main_iters_during=len(during),
               main_iter_max_during_ms=round(1e3 * max(during or [0]), 2),
               main_iter_median_before_ms=round(1e3 * before[len(before) // 2], 3))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    if sys.argv[1:] == ["after-kill"]:
        for threaded in (False, True):     # each in a fresh process, each after its own kill
            subprocess.run([sys.executable, os.path.abspath(__file__), "_child", str(int(threaded))], check=True)
    elif sys.argv[1:2] == ["_child"]:
        main(after_kill=True, threaded=sys.argv[2] == "1")
    else:
        main(threaded=False)
        main()
