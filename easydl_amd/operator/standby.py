"""Hot-standby role processes (SURVEY.md §5.3 "hot-standby processes ... remove
the multi-second Python/torch import from TTR", §7.3 hard part 3; the capability is the
reference's "recover failed parameter servers and workers and resume the training",
/root/reference/README.md:25-29, and the operator's replace-a-Pod flow,
/root/reference/docs/design/elastic-training-operator.md:97-101).

A standby is started by the local ElasticOperator ahead of any failure as
``python -m easydl_amd.operator.standby``.  It pays every start-up cost that
does not depend on WHICH role it will become:

* imports torch and the framework (trainer, models, comm, checkpoint, PS) —
  not the job's entry module itself, whose top level may start training;
* loads the gfx950 kernel library (code-object registration) and initialises
  the HIP runtime (device enumeration) without creating a context on any GPU —
  the GPU is chosen at takeover (``EDL_GPU``), so one spare covers any rank;

then parks on the job store.  With ``EDL_STANDBY_PREMAP=1`` it also maps and
pre-faults the job's snapshot segments while parked (restore 4.9 -> 4.0 s for
96 GB on one MI355X), but in that run the killed worker's exit, which unpins
the same pages, took 6.4 s instead of ~2.5 s, so it is off by default.  When a role process dies the operator writes
``standby/assign/<standby name>`` = ``{"env": {...}, "argv": [...]}``; the
standby applies the environment (role, index, generation, GPU, CU/HBM plan),
sets ``sys.argv`` and runs the role's module in-process with ``runpy`` — it
becomes ``<job>-<role>-<index>`` without a new process (its pid is the new
incarnation's pid, so exit events keep flowing through the supervisor).
"""
from __future__ import annotations

import gc
import importlib
import json
import os
import runpy
import sys
import threading
import time


def module_of(argv: list[str]) -> str | None:
    """The module of a ``python -m <module> ...`` command, else None (not runnable by a standby)."""
    if len(argv) >= 3 and os.path.basename(argv[0]).startswith("python") and argv[1] == "-m":
        return argv[2]
    return None


PREWARM_MODULES = ("easydl_amd.trainer.elastic", "easydl_amd.ckpt.manager", "easydl_amd.models.llama",
                   "easydl_amd.parallel.tp", "easydl_amd.trainer.ps_trainer", "easydl_amd.trainer.data")


def prewarm() -> dict:
    t0 = time.perf_counter()
    import torch  # noqa: F401

    from easydl_amd import _native
    for m in PREWARM_MODULES:
        importlib.import_module(m)
    out = {"import_s": round(time.perf_counter() - t0, 3)}
    if _native.kernels_available():
        out["kernels"] = True
    n = torch.cuda.device_count()
    out["gpus"] = n
    if n:
        torch.cuda.init()  # HIP runtime + device enumeration; contexts stay lazy (per device, at takeover)
    out["prewarm_s"] = round(time.perf_counter() - t0, 3)
    return out


def _llama_warm_bytes(cfg, tokens: int) -> int:
    """Rough peak of a one-layer forward/backward: bf16 weights + gradients, activations, logits."""
    kv = cfg.dim // cfg.n_heads * cfg.n_kv_heads
    layer = cfg.dim * (2 * cfg.dim + 2 * kv) + 3 * cfg.dim * cfg.ffn_dim
    params = cfg.vocab_size * cfg.dim * (1 if cfg.tie_embeddings else 2) + cfg.n_layers * layer
    return 4 * params + tokens * (10 * cfg.vocab_size + 64 * cfg.dim + 16 * cfg.ffn_dim)


WARM_INFO: dict = {}     # what the last warm_device did (logged by the standby)
WARM_STREAMS: dict = {}  # GPU -> the stream its warm-up ran on (the replacement's trainer keeps it)


def _warm_llama(dev, spec: dict, info: dict | None = None) -> bool:
    """Forward + backward of one layer of the worker's model at its micro-batch shape, with its
    parameters in flat buffers as the trainer has them (parallel/flat.py: weight gradients are
    GEMMs accumulating into the flat gradient buffer, a different hipBLASLt solution than a
    plain ``.grad``): the GEMM shapes, attention and norm kernels of the real step.  Skipped
    when the GPU has not got twice the memory it needs free."""
    import torch

    from easydl_amd.models.llama import Llama, LlamaConfig
    fields = LlamaConfig.__dataclass_fields__
    cfg = LlamaConfig(**{k: v for k, v in spec.get("cfg", {}).items() if k in fields})
    cfg.n_layers = 1
    b, s = (int(x) for x in spec["batch"])
    free, _ = torch.cuda.mem_get_info(dev)
    need = _llama_warm_bytes(cfg, b * s)
    wi = WARM_INFO if info is None else info
    wi.update(free_gb=round(free / 2**30, 1), need_gb=round(need / 2**30, 1))
    if free < 2 * need + (4 << 30):
        # Not room for the micro-batch shape: still run the layer at the worker's widths on a
        # short sequence.  The GEMM solutions for the real M differ, but hipBLASLt's library,
        # the attention / norm / loss kernels at these widths and their code objects are then
        # loaded HERE, while HBM is calm, not in the replacement's first step.  (It does not
        # prevent the third-takeover crash of profiles/r06_three_failures_8b.md; a one-sequence
        # warm-up at 8k tokens did not either.)
        b, s = 1, min(s, 512)
        need = _llama_warm_bytes(cfg, b * s)
        if free < 2 * need + (4 << 30) or os.environ.get("EDL_STANDBY_WARM_SHORT", "1") == "0":
            return False
        wi["reduced_tokens"] = b * s
    from easydl_amd.parallel.flat import FlatParams
    model = Llama(cfg, device=dev)
    flat = FlatParams(model)
    ids = torch.randint(0, cfg.vocab_size, (b, s), device=dev)
    model(ids, ids).backward()
    torch.cuda.synchronize(dev)
    del model, flat, ids
    gc.collect()    # the flat buffers' gradient hooks form reference cycles with the parameters
    return True


def warm_device(gpu: int, spec: dict | None = None, set_stream: bool = False, info: dict | None = None) -> float:
    """One forward + backward + optimizer step of a small Llama of head dim 128 on ``gpu``,
    preceded, when the worker published its shape (``spec``, ElasticTrainer._publish_warm_spec),
    by a forward + backward of one layer of its model at full width.

    A fresh process's first training step pays ~0.8 s of first-use costs on the host:
    code-object loads of this framework's kernels and of the PyTorch kernels the model uses,
    hipBLASLt initialisation, allocator growth (scripts/first_step_probe.py: first step
    1.21 s cold, 0.41 s after a warm-up).  A parked standby that already holds a context on
    the GPU (it mapped the workers' HBM there, utils/vram.py) pays most of that up front, so
    the replacement's first step -- the last phase of its time-to-recover -- does not.  The
    small model covers the optimizer and the framework's kernels; the full-width layer covers
    the shape-dependent part (GEMM solutions, 1.21 s -> 0.41 s in the probe).  Its memory is
    freed before this returns.  Returns seconds."""
    import torch

    from easydl_amd.models.llama import Llama, LlamaConfig
    from easydl_amd.optim import FlatAdamW
    from easydl_amd.parallel.flat import FlatParams
    from easydl_amd.ops import gemm_tuning
    t0 = time.perf_counter()
    dev = torch.device("cuda", gpu)
    # the replacement's GEMMs run through TunableOp with the shipped selections
    # (ElasticTrainer.__init__) on a non-default stream: warm up in the same configuration,
    # on the stream the trainer will then keep using (``set_stream``: a per-stream hipBLASLt
    # workspace; the process's current stream stays set)
    gemm_tuning.apply()
    if set_stream and torch.cuda.current_stream(dev).cuda_stream == 0:
        # (the current stream is per thread: a warm-up thread records it for the takeover)
        WARM_STREAMS[gpu] = torch.cuda.Stream(dev)
        torch.cuda.set_stream(WARM_STREAMS[gpu])
    cfg = LlamaConfig(vocab_size=1024, dim=512, n_layers=1, n_heads=4, n_kv_heads=2, ffn_dim=1024, max_seq_len=256)
    wi = WARM_INFO if info is None else info
    with torch.cuda.device(dev):
        wi.clear()
        if spec and spec.get("model") == "llama":
            t1 = time.perf_counter()
            wi["full_width"] = _warm_llama(dev, spec, wi)
            wi["full_width_s"] = round(time.perf_counter() - t1, 3)
        model = Llama(cfg, device=dev)
        flat = FlatParams(model)
        opt = FlatAdamW(flat)
        ids = torch.randint(0, cfg.vocab_size, (2, 256), device=dev)
        loss = model(ids, ids)
        loss.backward()
        opt.step()
        torch.cuda.synchronize(dev)
        del model, flat, opt, loss, ids
        gc.collect()    # (see _warm_llama): otherwise the state stays allocated until a GC cycle
        # this GPU's cache only: a global empty_cache from a late warm-up thread would drop the
        # slab already reserved on another GPU (_reserve_slab)
        _release_device_cache(dev.index if dev.index is not None else torch.cuda.current_device())
    return time.perf_counter() - t0


def _warm_one(kv, name: str, gpu: int, spec) -> None:
    """Warm-up of one GPU (a thread of the parked standby); its key tells the worker it is done."""
    info: dict = {}
    try:
        s = round(warm_device(gpu, spec, set_stream=True, info=info), 3)
        info = dict(s=s, spec=spec is not None, **info)
        kv.set(f"standby/warm/{name}/gpu{gpu}", json.dumps(info))
        print(f"standby {name}: warm-up on GPU {gpu}: {json.dumps(info)}", file=sys.stderr, flush=True)
    except Exception as e:  # noqa: BLE001 - an optimisation only
        print(f"standby: warm-up on GPU {gpu} failed: {e}", file=sys.stderr)
        kv.set(f"standby/warm/{name}/gpu{gpu}", json.dumps({"error": str(e)[:200]}))


SLABS: dict = {}   # GPU -> bytes of HBM this parked standby holds reserved in its caching allocator


def _reserve_slab(kv, name: str, gpu: int, slot: str) -> None:
    """Once ``slot``'s worker has run its first step (it published its step's HBM need): reserve
    what the GPU still has free, less a margin the worker keeps for itself, in THIS process's
    caching allocator on the stream the replacement will compute on (WARM_STREAMS) -- allocated
    and freed, so it stays cached.

    Why: a replacement's first step allocates its activations right after the dead worker died,
    and fresh HBM is slow to hand out then (the r06 drill: 0.8-2.7 s per micro-batch that needed
    new segments vs 0.35-0.7 s steady; profiles/r06_ttr_first_step.md).  Blocks carved from a
    slab reserved while everything was calm cost nothing.  The slab is at most the worker's
    published need, and ``EDL_STANDBY_SLAB_MARGIN_GB`` (default 12) stays free for the worker.
    ``EDL_STANDBY_SLAB=0`` turns it off."""
    import torch
    if os.environ.get("EDL_STANDBY_SLAB", "1") == "0" or gpu in SLABS:
        return
    from easydl_amd.utils import vram
    act, _, _ = vram.read_act(kv, slot)
    if not act:
        return
    dev = torch.device("cuda", gpu)
    margin = int(float(os.environ.get("EDL_STANDBY_SLAB_MARGIN_GB", 12)) * 2**30)
    free, _ = torch.cuda.mem_get_info(dev)
    want = min(act, free - margin) // (2 << 20) * (2 << 20)
    SLABS[gpu] = 0
    if want < (2 << 30):
        kv.set(f"standby/slab/{name}/gpu{gpu}", json.dumps({"gb": 0, "free_gb": round(free / 2**30, 1)}))
        return
    st = WARM_STREAMS.get(gpu)
    t0 = time.perf_counter()
    try:
        with torch.cuda.device(dev), torch.cuda.stream(st) if st is not None else _Null():
            buf = torch.empty(want, dtype=torch.uint8, device=dev)
            del buf
        SLABS[gpu] = want
    except RuntimeError as e:     # (out of memory: the worker grew meanwhile) -- an optimisation only
        print(f"standby {name}: slab of {want / 2**30:.1f} GB on GPU {gpu} failed: {e}", file=sys.stderr)
    kv.set(f"standby/slab/{name}/gpu{gpu}", json.dumps({"gb": round(SLABS[gpu] / 2**30, 1),
                                                        "free_gb": round(free / 2**30, 1),
                                                        "s": round(time.perf_counter() - t0, 3)}))
    print(f"standby {name}: GPU {gpu}: slab {SLABS[gpu] / 2**30:.1f} GB reserved ({free / 2**30:.1f} GB were "
          f"free) in {time.perf_counter() - t0:.3f} s", file=sys.stderr, flush=True)


def _release_device_cache(g: int) -> None:
    """Return ONE GPU's cached blocks to the driver.  ``torch.cuda.empty_cache()`` empties the
    caching allocator of every device -- at a takeover that would also drop the slab on the GPU
    the replacement is about to compute on, the very memory its first step needs.  An allocation
    larger than the device makes that device's allocator (and only it) free its cached blocks
    and retry before it gives up, which is the per-device release we want."""
    import torch
    try:
        torch.empty(2 * torch.cuda.get_device_properties(g).total_memory, dtype=torch.uint8,
                    device=torch.device("cuda", g))
    except torch.cuda.OutOfMemoryError:
        pass


def _release_slabs(keep: int | None) -> None:
    """Takeover of ``keep``'s GPU: the slabs on every other GPU go back to the driver; ``keep``'s
    stays cached for the replacement's first step."""
    for g in [g for g in SLABS if g != keep]:
        if SLABS.pop(g):
            _release_device_cache(g)


class _Null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def _import_vram(kv, held: dict) -> None:
    """Map (IPC) the state buffers every worker published; keep them referenced while parked."""
    from easydl_amd.utils import vram
    try:
        slots = vram.slots(kv)
    except Exception:  # noqa: BLE001
        return
    for slot in slots:
        try:
            held[slot] = vram.import_published(kv, slot, held.get(slot))
        except Exception as e:  # noqa: BLE001 - a worker mid-restart: try again next scan
            print(f"standby: vram import of {slot} failed: {e}", file=sys.stderr)
    # An exporter that died without this standby taking its place (a scale-down, another
    # spare took it, the job ended): let its HBM go back to the driver.
    now = time.monotonic()
    for slot, h in list(held.items()):
        if h is None or not vram.reaped(h.get("pid")):
            continue
        h.setdefault("dead_since", now)
        if now - h["dead_since"] > 10.0:
            del held[slot]


def _adopt_vram(held: dict, slot: str, kv, name: str) -> None:
    """Takeover of ``slot``: its dead predecessor's buffers back this process's state; every
    other worker's imports are released (they belong to live processes)."""
    from easydl_amd.utils import vram
    got = held.pop(slot, None)
    held.clear()
    if not got or not got.get("tensors"):
        return
    if not vram.dead(got.get("pid")):
        print(f"standby: {slot}'s exporter {got.get('pid')} is alive; not adopting", file=sys.stderr)
        return
    vram.adopt(got["tensors"], pid=got.get("pid"))
    kv.set(f"standby/vram/{name}", json.dumps({"slot": slot, "from": got.get("owner"),
                                               "tensors": len(got["tensors"])}))


def main() -> int:
    from easydl_amd.master.store import KV, make_tcp_store
    name = os.environ["EDL_STANDBY_NAME"]
    job = os.environ.get("EDL_JOB", "job")
    kv = KV(make_tcp_store(os.environ.get("EDL_MASTER_ADDR", "127.0.0.1"), int(os.environ["EDL_MASTER_PORT"]),
                           False), f"edl/{job}")
    info = prewarm()
    info.update(pid=os.getpid(), ts=time.time())
    kv.set(f"standby/ready/{name}", json.dumps(info))
    from easydl_amd.utils import vram
    if not info.get("gpus"):
        kv.set(f"standby/warm/{name}/cpu", json.dumps({}))   # nothing to warm on a CPU host
    elif not vram.enabled():
        kv.set(f"standby/warm/{name}/any", json.dumps({}))   # no hand-over: nothing per GPU
    key = f"standby/assign/{name}"
    premap = os.environ.get("EDL_STANDBY_PREMAP", "0") == "1"
    handoff = vram.enabled() and info.get("gpus", 0) > 0
    held: dict[str, dict] = {}     # worker slot -> imported state buffers (utils/vram.py)
    warmed: set[int] = set()       # GPUs this standby has run (or is running) its warm-up step on
    warming: list = []             # their warm-up threads
    late: dict = {}                # GPU -> warm spec, waiting for a window (its worker already trains)
    warm_thread: dict = {}         # GPU -> its warm-up thread (a slab is reserved once it is done)
    requested: set = set()         # GPUs of the window request filed
    req_id = 0
    warm_on = os.environ.get("EDL_STANDBY_WARMUP", "1") != "0"
    next_scan = next_vram = 0.0
    while True:
        a = kv.get(key)
        if a is not None:
            break
        if kv.exists("job/done"):
            return 0
        if handoff and time.monotonic() > next_vram:
            _import_vram(kv, held)
            next_vram = time.monotonic() + 0.25   # a worker waits for this warm-up before its first step
            for slot, h in sorted(held.items()):
                # (a worker's export may hold no tensors -- a replacement that itself adopted HBM
                # re-publishes only what it can: the warm-up of its GPU still applies)
                if not h or h["gpu"] in warmed:
                    continue
                if not warm_on:
                    warmed.add(h["gpu"])
                    kv.set(f"standby/warm/{name}/gpu{h['gpu']}", json.dumps({"warmup": "off"}))
                    continue
                published, spec = vram.read_warm(kv, slot)
                if not published:
                    continue            # the worker has not published its shape yet
                if vram.trained(kv, slot):
                    # that worker trains already (this standby is a refill after a takeover):
                    # warm up only in a window between two of its steps (utils/vram.py)
                    late[h["gpu"]] = spec
                    warmed.add(h["gpu"])
                    continue
                warmed.add(h["gpu"])
                # one thread per GPU: at N=8 every worker waits for its own GPU's warm-up before its
                # first step, and eight warm-ups in a row would hold the last one back ~8 x 1.3 s
                t = threading.Thread(target=_warm_one, args=(kv, name, h["gpu"], spec), daemon=True,
                                     name=f"warm-gpu{h['gpu']}")
                t.start()
                warming.append(t)
                warm_thread[h["gpu"]] = t
            for slot, h in sorted(held.items()):
                # the worker has trained a step and this GPU's warm-up is over: reserve the slab
                g = h["gpu"] if h else None
                if (g is not None and g in warmed and g not in SLABS and g not in late
                        and not (warm_thread.get(g) is not None and warm_thread[g].is_alive())):
                    _reserve_slab(kv, name, g, slot)
            if late and set(late) != requested:
                requested = set(late)
                req_id += 1
                vram.request_warm_window(kv, name, req_id, requested)
            for g in sorted(late):
                if kv.exists(f"standby/warm_grant/{name}/gpu{g}"):
                    t = threading.Thread(target=_warm_one, args=(kv, name, g, late.pop(g)), daemon=True,
                                         name=f"warm-gpu{g}")
                    t.start()
                    warming.append(t)
                    warm_thread[g] = t
                    SLABS.pop(g, None)     # (its warm-up empties the cache: reserve again after it)
        if premap and time.monotonic() > next_scan:
            from easydl_amd.ckpt.manager import premap_job_segments
            mapped = premap_job_segments(job)
            if mapped:
                kv.set(f"standby/premapped/{name}", json.dumps(mapped))
            next_scan = time.monotonic() + 2.0
        time.sleep(0.005)
    for t in warming:   # a takeover right after start-up: let the warm-ups finish first
        t.join()
    kv.delete(f"standby/warm_req/{name}")
    a = a if isinstance(a, dict) else json.loads(a)
    os.environ.update({k: str(v) for k, v in a["env"].items()})
    gpu = a["env"].get("EDL_GPU")
    if gpu is not None and int(gpu) in WARM_STREAMS:
        import torch
        torch.cuda.set_stream(WARM_STREAMS[int(gpu)])   # the stream the warm-up ran on (its hipBLASLt workspace)
    if SLABS:
        _release_slabs(int(gpu) if gpu is not None else None)   # this GPU's slab feeds the first step
    # the parked loop's variables still name the imported state ("h" is the last slot's record,
    # "t" a warm-up thread): this frame lives as long as the role it runs, so without this the
    # dead worker's HBM would stay mapped after the trainer re-homed its state into its own
    # memory -- 120 GB at Llama-3-8B, and the next step ran out of memory
    h = t = None  # noqa: F841
    if handoff:
        _adopt_vram(held, f"worker{a['env'].get('EDL_INDEX', '')}", kv, name)
    held.clear()
    warming.clear()
    late.clear()
    gc.collect()
    argv = a["argv"]
    mod = module_of(argv)
    if mod is None:
        print(f"standby {name}: cannot run {argv!r} in-process", file=sys.stderr)
        return 3
    sys.argv = [mod] + argv[3:]
    kv.set(f"standby/taken/{name}", json.dumps({"as": a["env"].get("EDL_INDEX"), "ts": time.time()}))
    runpy.run_module(mod, run_name="__main__", alter_sys=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
