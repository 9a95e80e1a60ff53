"""Scale-up mid-run benchmark (BASELINE.json config 2: "ResNet-50 bf16 elastic
DDP, scale 1->8 MI355X mid-run (RCCL re-init)").

Runs a real job through the local ElasticOperator: ``--start`` workers train
ResNet-50 (bf16, channels-last, synthetic images; a small ResNet on CPU);
after ``--scale-step`` committed steps the driver raises the JobResource's
worker replicas to ``--end`` (what ``edl scale`` / the Brain's re-plan do).
The operator spawns the new workers, the rendezvous forms a larger epoch at
the next step boundary, survivors broadcast the state to the joiners and
everyone builds the new RCCL communicator — no surviving process restarts.

Reports images/s per world size and the scale-up latency breakdown (spawn ->
joined -> epoch formed -> comm ready -> state synced -> first step at the new
size) from the merged event timeline.  Prints one JSON line.

    python -m easydl_amd.trainer.scale_bench --start 1 --end 8 --steps 30
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
import tempfile
import threading
import time

from easydl_amd.utils.events import read_events


def _gpus() -> list[int]:
    from easydl_amd.brain.collectors import kfd_gpus
    return [g.index for g in kfd_gpus()]


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--start", type=int, default=1)
    ap.add_argument("--end", type=int, default=8)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--scale-step", type=int, default=10)
    ap.add_argument("--batch", type=int, default=256, help="per-worker images per step")
    ap.add_argument("--share-gpu", action="store_true",
                    help="every worker on GPU 0 with the xGMI engine as the only data plane (RCCL refuses "
                         "two ranks on one device): the scale-up path measured on a single MI355X")
    a = ap.parse_args(argv)
    from easydl_amd.api.spec import ElasticJob, JobResource, Resource, RoleResource
    from easydl_amd.operator.reconciler import ElasticOperator, OperatorConfig
    gpus = _gpus()
    share = a.share_gpu and bool(gpus)
    if share:
        gpus = [gpus[0]] * a.end
    end = min(a.end, len(gpus)) if gpus else a.end
    run_dir = tempfile.mkdtemp(prefix="edl-scale-", dir=os.environ.get("EDL_SCALE_DIR", None))
    cpu_batch = 4
    per = a.batch if gpus else cpu_batch
    gb = per * end   # global batch fixed across the resize: 1 worker accumulates end micro-batches
    env = {"EDL_SCALE_STEPS": str(a.steps), "EDL_SCALE_BATCH": str(per), "EDL_SCALE_GB": str(gb)}
    if share:
        env["EDL_COMM"] = "xgmi-only"
        env["EDL_XGMI_MAX_BLOCKS"] = "16"   # all ranks' engine grids must be co-resident on the one GPU
    job = ElasticJob(name="scale", command="python -m easydl_amd.trainer.scale_bench --worker", env=env,
                     min_workers=1, max_workers=end)
    jr = JobResource("scale-resource", "scale", {"worker": RoleResource(a.start, Resource(gpu=1 if gpus else 0,
                                                                                         cpu=2))})
    op = ElasticOperator(job, run_dir, cfg=OperatorConfig(gpus=gpus[:end], cpus=[]), job_resource=jr)
    scaled = {}

    def scaler():
        # wait for the scale step, then raise the replicas (what `edl scale` writes)
        t_end = time.time() + 900
        while time.time() < t_end and not op.done:
            evs = read_events(run_dir)
            steps = [e["step"] for e in evs if e["kind"] == "step_done"]
            if steps and max(steps) >= a.scale_step and op.kv is not None:
                cur = JobResource.from_dict(json.loads(op.kv.get_str("jobresource")))
                cur.roles["worker"].replicas = end
                cur.version += 1
                scaled["ts"] = time.time()
                op.kv.set("jobresource", json.dumps(cur.to_dict()))
                return
            time.sleep(0.2)

    th = threading.Thread(target=scaler, daemon=True)
    th.start()
    rc = op.run(timeout_s=1200)
    ev = read_events(run_dir)
    done = [e for e in ev if e["kind"] == "step_done" and e.get("proc") == "worker0"]
    per_world: dict[int, list[float]] = {}
    for prev, cur in zip(done, done[1:]):
        if prev.get("world") == cur.get("world"):
            per_world.setdefault(cur["world"], []).append(cur["ts"] - prev["ts"])
    ips = {w: round(gb / sorted(v)[len(v) // 2], 1) for w, v in per_world.items() if v}
    t0 = scaled.get("ts")

    def first(kind, pred=lambda e: True):
        e = next((e for e in ev if t0 and e["ts"] >= t0 and e["kind"] == kind and pred(e)), None)
        return None if e is None else round(e["ts"] - t0, 3)

    new_world = lambda e: e.get("world") == end  # noqa: E731
    out = {"metric": "elastic scale-up mid-run (ResNet-50 bf16 DDP)" if gpus else "elastic scale-up (CPU ResNet)",
           "start": a.start, "end": end, "global_batch": gb, "images_per_s_by_world": ips, "operator_rc": rc,
           "n_gpus": (1 if share else end) if gpus else 0, "shared_gpu": share,
           "comm": env.get("EDL_COMM", os.environ.get("EDL_COMM", "pg")),
           "scale_up_s": {"spawn": first("spawn", lambda e: e.get("role") == "worker"), "joined": first("joined"),
                          "epoch_formed": first("epoch_formed", new_world),
                          "comm_ready": first("comm_ready", new_world),
                          "state_synced": first("state_synced"), "first_step": first("step_done", new_world)}}
    print(json.dumps(out), flush=True)
    if os.environ.get("EDL_SCALE_KEEP") != "1":
        shutil.rmtree(run_dir, ignore_errors=True)
    return 0 if rc == 0 and ips else 1


def worker() -> None:
    import torch

    from easydl_amd.models.resnet import ResNet, SyntheticImages, resnet50
    from easydl_amd.trainer.elastic import ElasticTrainer
    e = os.environ
    cuda = torch.cuda.is_available()
    batch = int(e.get("EDL_SCALE_BATCH", 256))
    if cuda:
        model_fn, data = (lambda d: resnet50(d)), SyntheticImages()
    else:
        model_fn = lambda d: ResNet(layers=(1, 1, 1, 1), num_classes=10, width=8).to(d)  # noqa: E731
        imgs = SyntheticImages(size=32, classes=10)

        class _F32:  # fp32 images for the CPU stand-in
            def __len__(self):
                return len(imgs)

            def batch(self, idx, device="cpu"):
                return imgs.batch(idx, device, dtype=torch.float32)

        data = _F32()
    # fixed global batch: the 1-worker phase accumulates, the scaled phase splits it
    tr = ElasticTrainer(model_fn, global_batch=int(e["EDL_SCALE_GB"]), micro_batch=batch, lr=0.1,
                        optimizer="sgd", weight_decay=1e-4)
    tr.fit(lambda m, b: m(*b), data, num_steps=int(e.get("EDL_SCALE_STEPS", 30)))
    tr.close()


if __name__ == "__main__":
    if "--worker" in sys.argv:
        worker()
    else:
        sys.exit(main())
