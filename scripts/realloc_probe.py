"""How long does HBM allocation take right after a process holding most of the
GPU was SIGKILLed mid-work?  (TTR of a 1-GPU restart: the replacement's model
build was 25x slower than a cold start's.)

    python scripts/realloc_probe.py            # victim, then probes at several delays
"""
import json
import os
import signal
import subprocess
import sys
import time


def victim():
    import torch
    x = torch.empty(int(180e9), dtype=torch.uint8, device="cuda")
    a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
    torch.cuda.synchronize()
    print("ready", flush=True)
    while True:
        for _ in range(50):
            a = a @ a
            a = a / a.norm()
        x[:1024].fill_(1)


def probe():
    import torch
    t0 = time.perf_counter()
    torch.empty(1, device="cuda")
    t1 = time.perf_counter()
    bufs = [torch.empty(int(16e9), dtype=torch.uint8, device="cuda") for _ in range(8)]
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    for b in bufs:
        b.fill_(0)
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    print(json.dumps({"ctx_s": round(t1 - t0, 3), "alloc128g_s": round(t2 - t1, 3), "fill_s": round(t3 - t2, 3)}),
          flush=True)


def main():
    if sys.argv[1:] == ["victim"]:
        return victim()
    if sys.argv[1:] == ["probe"]:
        return probe()
    subprocess.run([sys.executable, __file__, "probe"], check=True, timeout=120)  # cold baseline
    for delay in (0.0, 3.0, 8.0):
        v = subprocess.Popen([sys.executable, __file__, "victim"], stdout=subprocess.PIPE, text=True)
        assert v.stdout.readline().strip() == "ready"
        time.sleep(2.0)
        t0 = time.perf_counter()
        os.kill(v.pid, signal.SIGKILL)
        v.wait()
        t_exit = time.perf_counter() - t0
        time.sleep(delay)
        print(json.dumps({"delay_after_exit_s": delay, "victim_exit_s": round(t_exit, 3)}), flush=True)
        subprocess.run([sys.executable, __file__, "probe"], check=True, timeout=120)


if __name__ == "__main__":
    main()
