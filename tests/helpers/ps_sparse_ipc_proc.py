"""Processes of the row-sparse GPU-transport test: 2 PS (dense shard + embedding stripes in
HBM) and DeepFM workers, all on one GPU (IPC mapping, peer reads / writes and the inbox
protocol run exactly as across GPUs).

argv: ps <index> <port_file> | worker <port0> <port1> <wid> <steps> <out> | check <port0> <port1> <out>

The worker counts every ``Tensor.cpu()`` / ``.tolist()`` / ``.item()`` issued inside its
training steps: the GPU sparse path (device-side owner split, gather from the mapped
stripes, scatter into the PS's sparse inboxes, event-ordered push) must issue none."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from easydl_amd.models.deepctr import DeepFM, SyntheticCTR, auc  # noqa: E402
from easydl_amd.ps.client import PSClient, shard_of  # noqa: E402
from easydl_amd.ps.embedding import table_shard_spec  # noqa: E402
from easydl_amd.ps.server import ParameterServer  # noqa: E402

VOCAB, HIDDEN = 1000, (128, 128)
role = sys.argv[1]
torch.manual_seed(0)
data = SyntheticCTR(60000, vocab=VOCAB)


def ref_model(device=None):
    return DeepFM(vocab=VOCAB, hidden=HIDDEN, device=device)


if role == "ps":
    idx, pf = int(sys.argv[2]), sys.argv[3]
    ref = ref_model()
    ps = ParameterServer(idx, shard_of(ref, 2, idx), lr=2e-3, device="cuda", tables=table_shard_spec(ref, 2, idx),
                         sparse_optimizer="adagrad", sparse_lr=0.05).start()
    with open(pf + ".tmp", "w") as f:
        f.write(str(ps.port))
    os.replace(pf + ".tmp", pf)
    while not os.path.exists(pf + ".stop"):
        time.sleep(0.05)
    with open(pf + ".steps", "w") as f:
        json.dump({n: t.step for n, t in ps.tables.items()}, f)
    ps.stop()
elif role == "worker":
    ports = [int(sys.argv[2]), int(sys.argv[3])]
    wid, steps, out = int(sys.argv[4]), int(sys.argv[5]), sys.argv[6]
    m = ref_model("cuda")
    c = PSClient(2, lambda i: ("127.0.0.1", ports[i]), f"w{wid}", transport="ipc")
    c.bind(m)
    host_reads = {"n": 0}
    orig = {k: getattr(torch.Tensor, k) for k in ("cpu", "tolist", "item")}

    def counting(name):
        def f(self, *a, **k):
            host_reads["n"] += 1
            return orig[name](self, *a, **k)
        return f
    batches = [data.batch(range(b0, b0 + 256), "cuda") for b0 in
               ((step * 2 + wid) * 256 % 50000 for step in range(steps))]   # data staged before the loop
    c.pull(m)
    for k in orig:
        setattr(torch.Tensor, k, counting(k))
    try:
        for step in range(steps):
            m.zero_grad()
            m(*batches[step]).backward()
            c.push(m, step, then_pull=True)
    finally:
        for k, f in orig.items():
            setattr(torch.Tensor, k, f)
    torch.cuda.synchronize()
    with open(out, "w") as f:
        json.dump({"wid": wid, "versions": c.versions, "host_reads": host_reads["n"], "paths": c.sparse_path}, f)
else:  # check: evaluate the trained tables through the TCP path (CPU split) and the IPC gather
    ports, out = [int(sys.argv[2]), int(sys.argv[3])], sys.argv[4]
    a, b = ref_model("cuda"), ref_model("cuda")
    ca = PSClient(2, lambda i: ("127.0.0.1", ports[i]), "ca", transport="ipc")
    cb = PSClient(2, lambda i: ("127.0.0.1", ports[i]), "cb", transport="tcp")
    ca.bind(a)
    cb.bind(b)
    ca.pull(a)
    cb.pull(b)
    ids = torch.randint(0, 26 * VOCAB, (4096,), device="cuda")
    ra, rb = ca.pull_rows("emb", ids), cb.pull_rows("emb", ids)
    a.eval()
    with open(out, "w") as f:
        json.dump({"rows_equal": bool(torch.equal(ra, rb)), "auc": auc(a, data, device="cuda"),
                   "paths_a": ca.sparse_path, "paths_b": cb.sparse_path}, f)
