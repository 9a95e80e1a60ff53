"""One rank of a TP=2 Llama (bf16, HIP kernels) whose tensor-parallel collectives
all run on the hand-written xGMI engine (Communicator(data_backend="xgmi"):
SUM / MAX all-reduce, and all-gather / reduce-scatter with SP=1), compared with
the dense fp32 model on the CPU.  Both ranks share one GPU, which the engine's
IPC mapping and flag protocol treat exactly like two GPUs of a node."""
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
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
store = dist.TCPStore("127.0.0.1", int(os.environ["PORT"]), world, rank == 0, timeout=datetime.timedelta(seconds=60))
comm = Communicator(store, rank, world, 1, device=dev, job="tpx", timeout_s=30.0, data_backend="xgmi")
cfg = get_config("llama-tiny", n_layers=2, dim=512, n_heads=4, n_kv_heads=2, ffn_dim=1024, vocab_size=1024)
torch.manual_seed(0)
dense = Llama(cfg, dtype=torch.float32)
for p_ in dense.parameters():   # bf16-representable weights: both models start from the same values
    p_.data = p_.data.bfloat16().float()
ids = torch.randint(0, cfg.vocab_size, (2, 128))
labels = torch.randint(0, cfg.vocab_size, (2, 128))
loss_d = dense(ids, labels)
loss_d.backward()
g = TPGroup(comm, sequence_parallel=os.environ.get("SP") == "1")
tp = LlamaTP(cfg, g, device=dev, dtype=torch.bfloat16)
sd = shard_state_dict({k: v.detach() for k, v in dense.named_parameters()}, cfg, rank, world)
with torch.no_grad():
    for n, p_ in tp.named_parameters():
        p_.copy_(sd[n])
loss_t = tp(ids.to(dev), labels.to(dev))
loss_t.backward()
tp.sync_sp_grads()
torch.cuda.synchronize()
dgrads = shard_state_dict({k: v.grad for k, v in dense.named_parameters()}, cfg, rank, world)
err = max((p_.grad.float().cpu() - dgrads[n]).abs().max().item() / (dgrads[n].abs().max().item() + 1e-9)
          for n, p_ in tp.named_parameters())
res = {"loss_d": loss_d.item(), "loss_t": loss_t.item(), "grad_rel_err": err, "backend": comm.backend,
       "healthy": comm.healthy()}
json.dump(res, open(os.environ["OUT"] + f".{rank}", "w"))
print(json.dumps(res), flush=True)
comm.ctrl_barrier() if hasattr(comm, "ctrl_barrier") else None
comm.xgmi.close()
