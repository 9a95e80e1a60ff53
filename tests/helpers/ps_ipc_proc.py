"""Processes of the PS GPU-transport test (all on one GPU: IPC mapping, peer
copies and the inbox protocol run exactly as across GPUs).

argv: ps <port_file> | worker <port> <wid> <steps> | check <port> <out>"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from easydl_amd.models.mlp import MLP, SyntheticMNIST, accuracy  # noqa: E402
from easydl_amd.ps.client import PSClient, shard_of  # noqa: E402
from easydl_amd.ps.server import ParameterServer  # noqa: E402

role = sys.argv[1]
torch.manual_seed(0)
data = SyntheticMNIST(6000)
if role == "ps":
    ref = MLP()
    ps = ParameterServer(0, shard_of(ref, 1, 0), lr=3e-3, device="cuda").start()
    with open(sys.argv[2], "w") as f:
        f.write(str(ps.port))
    while not os.path.exists(sys.argv[2] + ".stop"):
        time.sleep(0.05)
    ps.stop()
elif role == "worker":
    port, wid, steps = int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    m = MLP(device="cuda", dtype=torch.bfloat16)
    c = PSClient(1, lambda i: ("127.0.0.1", port), f"w{wid}", transport="ipc")
    c.bind(m)
    for step in range(steps):
        if step == 0 or wid % 2:   # odd workers: separate pull; even: push + pull in one message
            c.pull(m)
        m.zero_grad()
        b0 = (step * 2 + wid) * 32 % 5000
        x, y = data.batch(range(b0, b0 + 32), "cuda")
        m(x.bfloat16(), y).backward()
        c.push(m, step, then_pull=(wid % 2 == 0))
    print(json.dumps({"wid": wid, "versions": c.versions}))
else:  # check: IPC pull (bf16 via the HIP kernel) == TCP pull (fp32 -> bf16) bit for bit
    port = int(sys.argv[2])
    a = MLP(device="cuda", dtype=torch.bfloat16)
    b = MLP(device="cuda", dtype=torch.bfloat16)
    ca = PSClient(1, lambda i: ("127.0.0.1", port), "ca", transport="ipc")
    cb = PSClient(1, lambda i: ("127.0.0.1", port), "cb", transport="tcp")
    ca.bind(a)
    cb.bind(b)
    va, vb = ca.pull(a), cb.pull(b)
    same = all(torch.equal(p, q) for p, q in zip(a.parameters(), b.parameters()))
    acc = accuracy(a.float(), data, device="cuda")
    with open(sys.argv[3], "w") as f:
        json.dump({"same": same, "va": va, "vb": vb, "acc": acc}, f)
