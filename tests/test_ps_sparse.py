"""Row-sparse PS ops (easydl_amd/ops/sparse.py, csrc/kernels/ps_sparse.hip).

CPU tier: the reference math equals a dense fp32 AdamW restricted to touched
rows (lazy Adam).  GPU tier: each HIP kernel against the fp32 PyTorch
reference of the same op, incl. duplicate and out-of-range ids."""
import math

import pytest
import torch

from easydl_amd.ops import sparse


def _dense_lazy_adam(w, m, v, ids, grad, lr, b1, b2, eps, wd, step):
    g = torch.zeros_like(w)
    g.index_add_(0, ids, grad)
    rows = torch.unique(ids)
    for r in rows.tolist():
        m[r] = b1 * m[r] + (1 - b1) * g[r]
        v[r] = b2 * v[r] + (1 - b2) * g[r] * g[r]
        denom = v[r].sqrt() / math.sqrt(1 - b2 ** step) + eps
        w[r] = w[r] * (1 - lr * wd) - lr / (1 - b1 ** step) * m[r] / denom


def test_segment_sum_and_lazy_adam_cpu():
    torch.manual_seed(0)
    rows, dim = 50, 8
    w = torch.randn(rows, dim)
    m, v = torch.zeros_like(w), torch.zeros_like(w)
    w2, m2, v2 = w.clone(), m.clone(), v.clone()
    w0 = w.clone()
    seen = torch.zeros(rows, dtype=torch.bool)
    for step in (1, 2, 3):
        ids = torch.randint(0, rows - 10, (40,))  # rows >= 40 are never touched
        seen[ids] = True
        grad = torch.randn(40, dim)
        uniq, comp = sparse.segment_sum_rows(ids, grad, rows)
        assert torch.equal(uniq, torch.unique(ids))
        sparse.sparse_rows_update(w, m, v, uniq, comp, kind="adam", lr=0.01, weight_decay=0.1, step=step)
        _dense_lazy_adam(w2, m2, v2, ids, grad, 0.01, 0.9, 0.999, 1e-8, 0.1, step)
    torch.testing.assert_close(w, w2, rtol=1e-5, atol=1e-6)
    assert torch.equal(w[~seen], w0[~seen]) and not m[~seen].any()  # lazy: untouched rows keep state


def test_gather_out_of_range_is_zero_cpu():
    t = torch.arange(24, dtype=torch.float32).view(6, 4)
    out = sparse.embed_gather(t, torch.tensor([1, -1, 7, 5]))
    assert torch.equal(out[0], t[1]) and torch.equal(out[3], t[5])
    assert not out[1].any() and not out[2].any()


@pytest.mark.gpu
def test_sparse_kernels_match_reference(cuda):
    torch.manual_seed(1)
    rows, dim, n = 1000, 128, 4096
    table = torch.randn(rows, dim)
    ids = torch.randint(-3, rows + 3, (n,))                  # duplicates and a few invalid ids
    grad = torch.randn(n, dim)
    # gather (fp32 and bf16 out)
    g_ref = sparse.embed_gather(table, ids)
    g_hip = sparse.embed_gather(table.cuda(), ids.cuda())
    torch.testing.assert_close(g_hip.cpu(), g_ref, rtol=0, atol=0)
    g16 = sparse.embed_gather(table.cuda(), ids.cuda(), out_dtype=torch.bfloat16)
    torch.testing.assert_close(g16.float().cpu(), g_ref.bfloat16().float(), rtol=0, atol=0)
    # segment sum (fp32 atomics: order-dependent rounding only)
    u_ref, c_ref = sparse.segment_sum_rows(ids, grad, rows)
    u_hip, c_hip = sparse.segment_sum_rows(ids.cuda(), grad.cuda(), rows)
    assert torch.equal(u_hip.cpu(), u_ref)
    torch.testing.assert_close(c_hip.cpu(), c_ref, rtol=1e-5, atol=1e-5)
    # lazy optimizers
    for kind in ("adam", "adagrad", "sgd"):
        w, m, v = table.clone(), torch.rand(rows, dim) * 0.1, torch.rand(rows, dim) * 0.1
        wg, mg, vg = w.cuda(), m.cuda(), v.cuda()
        sparse.sparse_rows_update(w, m, v, u_ref, c_ref, kind=kind, lr=1e-2, weight_decay=0.01, step=3)
        sparse.sparse_rows_update(wg, mg, vg, u_hip, c_hip, kind=kind, lr=1e-2, weight_decay=0.01, step=3)
        torch.cuda.synchronize()
        torch.testing.assert_close(wg.cpu(), w, rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(vg.cpu(), v, rtol=1e-5, atol=1e-5)
    # dense pull with cast
    src = torch.randn(1 << 20, device="cuda")
    dst = torch.empty(1 << 20, device="cuda", dtype=torch.bfloat16)
    sparse.pull_cast(src, dst)
    assert torch.equal(dst, src.bfloat16())


@pytest.mark.gpu
def test_deepfm_ps_shards_on_gpu(cuda):
    """PS shards (dense + embedding stripes) resident in HBM: pulls gather rows with
    the HIP kernel, pushes segment-sum + lazy Adagrad on the device."""
    import threading

    from easydl_amd.models.deepctr import DeepFM, SyntheticCTR, auc
    from easydl_amd.ps.client import PSClient, shard_of
    from easydl_amd.ps.embedding import table_shard_spec
    from easydl_amd.ps.server import ParameterServer
    torch.manual_seed(0)
    vocab = 1000
    data = SyntheticCTR(60000, vocab=vocab)
    ref = DeepFM(vocab=vocab, hidden=(128, 128))
    servers = [ParameterServer(i, shard_of(ref, 2, i), lr=2e-3, device="cuda", tables=table_shard_spec(ref, 2, i),
                               sparse_optimizer="adagrad", sparse_lr=0.05).start() for i in range(2)]
    assert servers[0].tables["emb"].w.is_cuda
    try:
        addrs = {i: (s.host, s.port) for i, s in enumerate(servers)}

        def work(wid):
            m = DeepFM(vocab=vocab, hidden=(128, 128), device="cuda")
            c = PSClient(2, lambda i: addrs[i], f"w{wid}")
            c.bind(m)
            for step in range(80):
                c.pull(m)
                m.zero_grad()
                b0 = (step * 2 + wid) * 256
                m(*data.batch(range(b0, b0 + 256), "cuda")).backward()
                c.push(m, step)
            c.close()

        ts = [threading.Thread(target=work, args=(w,)) for w in range(2)]
        [t.start() for t in ts]
        [t.join(120) for t in ts]
        m = DeepFM(vocab=vocab, hidden=(128, 128), device="cuda")
        c = PSClient(2, lambda i: addrs[i], "eval")
        c.bind(m)
        c.pull(m)
        assert auc(m, data, device="cuda") > 0.65
        assert servers[1].tables["emb"].step == 160
    finally:
        for s in servers:
            s.stop()


@pytest.mark.gpu
def test_ps_gpu_ipc_transport(cuda, tmp_path):
    """PS shard in HBM, two worker processes pulling through the mapped shard (HIP
    pull-cast kernel) and pushing into their inboxes; async updates all applied."""
    import json
    import os
    import subprocess
    import sys
    import time
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    helper = os.path.join(root, "tests", "helpers", "ps_ipc_proc.py")
    pf = str(tmp_path / "port")
    env = dict(os.environ, PYTHONPATH=root)
    ps = subprocess.Popen([sys.executable, helper, "ps", pf], env=env)
    try:
        t_end = time.time() + 60
        while not os.path.exists(pf) and time.time() < t_end:
            time.sleep(0.1)
        port = open(pf).read().strip()
        ws = [subprocess.Popen([sys.executable, helper, "worker", port, str(w), "60"], env=env,
                               stdout=subprocess.PIPE, text=True) for w in range(2)]
        outs = [w.communicate(timeout=120)[0] for w in ws]
        assert all(w.returncode == 0 for w in ws), outs
        out = str(tmp_path / "check.json")
        subprocess.run([sys.executable, helper, "check", port, out], env=env, check=True, timeout=120)
        r = json.load(open(out))
        assert r["same"], r          # IPC pull == TCP pull, bit for bit
        assert r["va"] == [120] and r["vb"] == [120]
        assert r["acc"] > 0.6, r
    finally:
        open(pf + ".stop", "w").close()
        ps.wait(timeout=30)


@pytest.mark.gpu
def test_ps_gpu_async_snapshot_restores_exactly(cuda):
    """HBM-resident PS shard snapshotted through the async engine (CU-masked copy stream,
    GPU checksum, fenced updates); a replacement PS restores it bit-exactly."""
    import os

    from easydl_amd import _native
    from easydl_amd.models.deepctr import DeepFM
    from easydl_amd.ps.client import shard_of
    from easydl_amd.ps.embedding import table_shard_spec
    from easydl_amd.ps.server import ParameterServer, PSSnapshotter
    torch.manual_seed(0)
    ref = DeepFM(vocab=200, hidden=(64, 64))
    snap = PSSnapshotter("snaptest", 0)
    ps = ParameterServer(0, shard_of(ref, 1, 0), lr=1e-2, device="cuda", tables=table_shard_spec(ref, 1, 0),
                         snapshot=snap, snapshot_every=3)

    def push():
        g = {n: torch.randn(ps.state.shapes[n]) for n in ps.state.names}
        g["sparse/emb/ids"] = torch.randint(0, 200 * 26, (64,))
        g["sparse/emb/grad"] = torch.randn(64, 16)
        ps._push("w", g)

    try:
        for _ in range(6):            # snapshots taken after versions 3 and 6
            push()
        expect = [b.clone() for b in ps.state_buffers()]
        push()                        # version 7: fenced behind the v6 copy
        assert _native.runtime()("edl_ckpt_wait", snap.engine, snap.ticket, 60000) == 1
        fresh = ParameterServer(0, shard_of(ref, 1, 0), lr=1e-2, device="cuda", tables=table_shard_spec(ref, 1, 0))
        assert PSSnapshotter("snaptest", 0).restore(fresh)
        assert fresh.version == 6
        assert all(torch.equal(a, b) for a, b in zip(fresh.state_buffers(), expect))
        assert not torch.equal(ps.state_buffers()[0], expect[0])   # the live shard moved on
    finally:
        for f in os.listdir("/dev/shm"):
            if f.startswith("edl-snaptest-ps"):
                os.unlink("/dev/shm/" + f)


@pytest.mark.gpu
def test_ps_sparse_push_during_inflight_snapshot(cuda):
    """Sparse-table rows pushed while a large snapshot is still copying are fenced
    behind it: the committed slot is the pre-push state and restores exactly."""
    import os

    from easydl_amd import _native
    from easydl_amd.models.deepctr import DeepFM
    from easydl_amd.ps.client import shard_of
    from easydl_amd.ps.embedding import table_shard_spec
    from easydl_amd.ps.server import ParameterServer, PSSnapshotter
    torch.manual_seed(0)
    vocab = 40000                      # 26 x 40k rows x 16 x fp32 x {w, m, v}: ~200 MB to copy
    ref = DeepFM(vocab=vocab, hidden=(64, 64))
    snap = PSSnapshotter("snapsp", 0)
    ps = ParameterServer(0, shard_of(ref, 1, 0), lr=1e-2, device="cuda", tables=table_shard_spec(ref, 1, 0),
                         snapshot=snap, snapshot_every=2)

    def push(n_ids):
        g = {n: torch.randn(ps.state.shapes[n]) for n in ps.state.names}
        g["sparse/emb/ids"] = torch.randint(0, vocab * 26, (n_ids,))
        g["sparse/emb/grad"] = torch.randn(n_ids, 16)
        ps._push("w", g)

    try:
        push(64)
        push(64)                      # version 2: snapshot enqueued, copy in flight
        expect = [b.clone() for b in ps.state_buffers()]
        push(1 << 16)                 # touches rows all over the table right away
        assert _native.runtime()("edl_ckpt_wait", snap.engine, snap.ticket, 60000) == 1
        fresh = ParameterServer(0, shard_of(ref, 1, 0), lr=1e-2, device="cuda", tables=table_shard_spec(ref, 1, 0))
        assert PSSnapshotter("snapsp", 0).restore(fresh)
        assert fresh.version == 2
        assert all(torch.equal(a, b) for a, b in zip(fresh.state_buffers(), expect))
    finally:
        for f in os.listdir("/dev/shm"):
            if f.startswith("edl-snapsp-ps"):
                os.unlink("/dev/shm/" + f)


@pytest.mark.gpu
def test_multi_tensor_push_pull_kernel(cuda):
    """edl_ps_multi_copy: one launch pushes scattered bf16 / fp32 gradients (and zeros
    for a missing one) into a flat fp32 buffer, and pulls it back with the cast."""
    from easydl_amd.ops.sparse import MultiCopyPlan
    torch.manual_seed(0)
    sizes = [1, 3, 4, 7, 1000, 4096 * 8 + 5, 65536 * 3 + 2]
    dts = [torch.bfloat16, torch.float32, torch.bfloat16, torch.float32, torch.bfloat16, torch.bfloat16,
           torch.float32]
    ts = [torch.randn(n, device=cuda).to(dt) for n, dt in zip(sizes, dts)]
    offs, o = [], 0
    for n in sizes + [16]:
        offs.append(o)
        o += (n + 3) // 4 * 4
    flat = torch.full((o,), 7.0, device=cuda)
    items = [(t, off, t.numel()) for t, off in zip(ts, offs)] + [(None, offs[-1], 16)]
    MultiCopyPlan(items, cuda).run(flat.data_ptr(), push=True)
    torch.cuda.synchronize()
    for t, off in zip(ts, offs):
        assert torch.equal(flat[off:off + t.numel()], t.float())
    assert torch.equal(flat[offs[-1]:offs[-1] + 16], torch.zeros(16, device=cuda))
    flat2 = torch.randn(o, device=cuda)
    outs = [torch.empty_like(t) for t in ts]
    MultiCopyPlan([(t, off, t.numel()) for t, off in zip(outs, offs)], cuda).run(flat2.data_ptr(), push=False)
    torch.cuda.synchronize()
    for t, off in zip(outs, offs):
        assert torch.equal(t, flat2[off:off + t.numel()].to(t.dtype))   # RNE cast, like .to()


@pytest.mark.gpu
def test_striped_gather_split_push_inbox_update_match_reference(cuda):
    """The GPU sparse-transport kernels against the host-split reference: a gather over P
    striped tables (pointer array), the device-side owner split into P inboxes, and the
    lazy update from an inbox whose row count lives on the device."""
    P, dim = 3, 16
    rows_global = 1000
    tabs = [torch.randn((rows_global - p + P - 1) // P, dim, device=cuda) for p in range(P)]
    tp = sparse.ptr_array(tabs, cuda)
    nr = torch.tensor([t.shape[0] for t in tabs], dtype=torch.int64, device=cuda)
    ids = torch.unique(torch.randint(0, rows_global, (700,), device=cuda))
    got = sparse.embed_gather_striped(tp, nr, ids, dim)
    want = torch.stack([tabs[int(i) % P][int(i) // P] for i in ids.cpu()])
    assert torch.equal(got, want)
    assert torch.equal(sparse.embed_gather_striped(tp, nr, ids, dim, out_dtype=torch.bfloat16), want.bfloat16())
    cap = 1024
    boxes = [(torch.full((cap,), -1, dtype=torch.int64, device=cuda), torch.zeros(cap, dim, device=cuda),
              torch.zeros(4, dtype=torch.int32, device=cuda)) for _ in range(P)]
    g = torch.randn(ids.numel(), dim, device=cuda)
    scratch = torch.zeros(8, dtype=torch.int32, device=cuda)
    sparse.sparse_split_push(ids, g, *(sparse.ptr_array([b[k] for b in boxes], cuda) for k in range(3)), cap, scratch)
    for p, (bi, bg, bc) in enumerate(boxes):
        k = int(bc[0])
        mine = (ids % P) == p
        assert k == int(mine.sum())
        order = torch.argsort(bi[:k])
        assert torch.equal(bi[:k][order], (ids[mine] // P).sort().values)
        assert torch.equal(bg[:k][order], g[mine][torch.argsort(ids[mine] // P)])
        # PS side: lazy Adagrad from the inbox == the host-count reference update
        w1, v1 = tabs[p].clone(), torch.rand_like(tabs[p])
        w2, v2 = w1.clone(), v1.clone()
        sparse.sparse_inbox_update(w1, None, v1, bi, bg, bc, kind="adagrad", lr=0.05, step=3)
        sparse.sparse_rows_update(w2, None, v2, bi[:k].contiguous(), bg[:k].contiguous(), kind="adagrad", lr=0.05,
                                  step=3)
        assert torch.equal(w1, w2) and torch.equal(v1, v2)


@pytest.mark.gpu
def test_deepfm_sparse_rows_over_ipc_no_host_copies(cuda, tmp_path):
    """elastic-deepctr-job on the GPU transport: 2 PS processes (dense shard + embedding
    stripes in HBM) and 2 DeepFM worker processes.  Rows are pulled by one gather over the
    mapped stripes and pushed by a device-side owner split into the PS's sparse inboxes;
    pushes are ordered by an interprocess event instead of a host sync.  No .cpu() /
    .item() / .tolist() in any training step; every sparse push and pull took the IPC
    path; the tables learn (AUC) and read back identically over TCP."""
    import json
    import os
    import subprocess
    import sys
    import time
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    helper = os.path.join(root, "tests", "helpers", "ps_sparse_ipc_proc.py")
    env = dict(os.environ, PYTHONPATH=root)
    pfs = [str(tmp_path / f"port{i}") for i in range(2)]
    pss = [subprocess.Popen([sys.executable, helper, "ps", str(i), pfs[i]], env=env) for i in range(2)]
    try:
        t_end = time.time() + 90
        while not all(os.path.exists(p) for p in pfs) and time.time() < t_end:
            time.sleep(0.1)
        ports = [open(p).read().strip() for p in pfs]
        outs = [str(tmp_path / f"w{w}.json") for w in range(2)]
        ws = [subprocess.Popen([sys.executable, helper, "worker", *ports, str(w), "60", outs[w]], env=env)
              for w in range(2)]
        assert [w.wait(timeout=180) for w in ws] == [0, 0]
        res = [json.load(open(o)) for o in outs]
        for r in res:
            assert r["host_reads"] == 0, r
            assert r["paths"]["ipc_pushes"] == 60 and r["paths"]["tcp_pushes"] == 0, r
            assert r["paths"]["ipc_pulls"] >= 120 and r["paths"]["tcp_pulls"] == 0, r
        chk = str(tmp_path / "check.json")
        subprocess.run([sys.executable, helper, "check", *ports, chk], env=env, check=True, timeout=120)
        c = json.load(open(chk))
        assert c["rows_equal"], c
        assert c["auc"] > 0.65, c
    finally:
        for p in pfs:
            open(p + ".stop", "w").close()
        for p in pss:
            p.wait(timeout=30)
    steps = json.load(open(pfs[1] + ".steps"))
    assert steps["emb"] == 120, steps       # every push of both workers applied
