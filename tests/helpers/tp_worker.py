"""TP=2 rank vs the dense model (gloo, CPU, fp32)."""
import datetime
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from easydl_amd.models.llama import Llama, get_config  # noqa: E402
from easydl_amd.parallel.comm import Communicator  # noqa: E402
from easydl_amd.parallel.tp import LlamaTP, TPGroup, shard_state_dict  # noqa: E402

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
torch.set_num_threads(1)
store = dist.TCPStore("127.0.0.1", int(os.environ["PORT"]), world, rank == 0, timeout=datetime.timedelta(seconds=60))
comm = Communicator(store, rank, world, 1, device="cpu", job="tp")
cfg = get_config("llama-tiny", n_layers=2, dim=64, n_heads=4, n_kv_heads=2, ffn_dim=128, vocab_size=128)
torch.manual_seed(0)
dense = Llama(cfg, dtype=torch.float32)
ids = torch.randint(0, 128, (2, 16))
labels = torch.randint(0, 128, (2, 16))
loss_d = dense(ids, labels)
loss_d.backward()
g = TPGroup(comm, sequence_parallel=os.environ.get("SP") == "1")
starts = [0]
_start = g.all_reduce_start


def counted_start(x):
    starts[0] += 1
    return _start(x)


g.all_reduce_start = counted_start
tp = LlamaTP(cfg, g, dtype=torch.float32)
sd = shard_state_dict({k: v.detach() for k, v in dense.named_parameters()}, cfg, rank, world)
with torch.no_grad():
    for n, p in tp.named_parameters():
        p.copy_(sd[n])
loss_t = tp(ids, labels)
loss_t.backward()
tp.sync_sp_grads()
dgrads = shard_state_dict({k: v.grad for k, v in dense.named_parameters()}, cfg, rank, world)
err = max((p.grad - dgrads[n]).abs().max().item() / (dgrads[n].abs().max().item() + 1e-9)
          for n, p in tp.named_parameters())
json.dump({"loss_d": loss_d.item(), "loss_t": loss_t.item(), "grad_rel_err": err, "overlap": tp.overlap,
           "async_starts": starts[0]},
          open(os.environ["OUT"] + f".{rank}", "w"))
comm.barrier()
