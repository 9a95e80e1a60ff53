"""Probe: can one process order its GPU stream after another process's GPU work
through an interprocess event (torch.cuda.Event(interprocess=True) ->
hipIpcGetEventHandle)?  Process A fills a shared tensor after ~50 ms of GPU work
and records the event; process B makes its stream wait on the imported event and
copies the tensor.  Prints one JSON line: supported / ordered."""
import json
import multiprocessing as mp
import sys


def producer(q_out, q_in):
    import torch
    from torch.multiprocessing.reductions import reduce_tensor
    torch.cuda.set_device(0)
    x = torch.zeros(1 << 24, device="cuda")
    ev = torch.cuda.Event(interprocess=True, enable_timing=False)
    ev.record()
    torch.cuda.synchronize()
    q_out.put((bytes(ev.ipc_handle()), reduce_tensor(x)[1]))
    q_in.get()                      # consumer is about to wait
    a = torch.randn(8192, 8192, device="cuda")
    for _ in range(20):
        a = a @ a * 1e-4             # ~ tens of ms of GPU work
    x.fill_(1.0)
    ev.record()
    q_out.put("recorded")
    q_in.get()
    torch.cuda.synchronize()


def consumer(q_in, q_out, res):
    import torch
    from torch.multiprocessing.reductions import rebuild_cuda_tensor
    torch.cuda.set_device(0)
    h, args = q_in.get()
    x = rebuild_cuda_tensor(*args)
    try:
        ev = torch.cuda.Event.from_ipc_handle(torch.device("cuda", 0), h)
    except Exception as e:  # noqa: BLE001
        res.put({"supported": False, "error": repr(e)[:300]})
        q_out.put("go")
        q_out.put("done")
        return
    q_out.put("go")
    assert q_in.get() == "recorded"
    s = torch.cuda.current_stream()
    s.wait_event(ev)
    y = x.clone()
    torch.cuda.synchronize()
    res.put({"supported": True, "ordered": bool((y == 1).all().item()), "ones": int((y == 1).sum().item())})
    q_out.put("done")


if __name__ == "__main__":
    ctx = mp.get_context("spawn")
    a2b, b2a, res = ctx.Queue(), ctx.Queue(), ctx.Queue()
    pa = ctx.Process(target=producer, args=(a2b, b2a))
    pb = ctx.Process(target=consumer, args=(a2b, b2a, res))
    pa.start()
    pb.start()
    out = res.get(timeout=120)
    pa.join(60)
    pb.join(60)
    print(json.dumps(out))
    sys.exit(0)
