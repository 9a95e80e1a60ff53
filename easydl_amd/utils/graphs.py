"""HIP graph replay for launch-bound, fixed-shape GPU work (evaluation / inference forwards).

A training step of the flagship models is GPU-bound (BERT-large fwd+bwd captured into one graph:
1.03x at batch 8, 1.00x at 32, profiles/r06_hip_graph_probe.md), so the trainer keeps eager
steps with their elastic hooks.  Forward-only work at small batch is the opposite: a few hundred
kernels of a few microseconds each, every one paying a host launch.  :class:`GraphedCallable`
captures ``fn(*tensors)`` once per input signature with stream capture (``torch.cuda.graph`` =
hipStreamBeginCapture .. hipGraphInstantiate on ROCm) and afterwards copies the inputs into the
captured buffers and replays the graph: one launch for the whole forward.  The hand-written HIP
kernels (``easydl_amd._native``) launch on the current stream and are captured like any other.

Rules of use: ``fn`` must not synchronise with the host or change shape with the data (no
``.item()``, no data-dependent allocation sizes); outputs are the captured buffers and are
overwritten by the next call (``clone()`` what must be kept); parameters are read in place, so
weight updates between calls (e.g. a new snapshot loaded by the evaluator) are seen by the next
replay.  Capture runs under ``torch.no_grad()`` unless ``grad=True``.
"""
from __future__ import annotations

import logging

import torch

log = logging.getLogger(__name__)


def _flat(out):
    if isinstance(out, torch.Tensor):
        return [out], lambda xs: xs[0]
    if isinstance(out, (tuple, list)):
        kind = type(out)
        return list(out), lambda xs: kind(xs)
    if isinstance(out, dict):
        keys = list(out)
        return [out[k] for k in keys], lambda xs: dict(zip(keys, xs))
    raise TypeError(f"GraphedCallable: unsupported output type {type(out).__name__}")


class GraphedCallable:
    """``g = GraphedCallable(fn); y = g(x1, x2)`` -- eager semantics, one graph launch per call
    for every input signature (shape, dtype, device) seen; at most ``max_graphs`` kept."""

    def __init__(self, fn, warmup: int = 2, grad: bool = False, max_graphs: int = 8):
        self.fn, self.warmup, self.grad, self.max_graphs = fn, warmup, grad, max_graphs
        self._graphs: dict = {}
        self._eager: set = set()      # input signatures whose capture failed
        self.captures = 0
        self.replays = 0

    def _eager_call(self, args):
        ctx = torch.enable_grad if self.grad else torch.no_grad
        with ctx():
            return self.fn(*args)

    def _capture(self, key, args):
        dev = args[0].device
        static = [a.detach().clone() for a in args]
        ctx = torch.enable_grad if self.grad else torch.no_grad
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side), ctx():
            for _ in range(self.warmup):   # library handles / workspaces / kernel code objects first
                self.fn(*static)
        torch.cuda.current_stream(dev).wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g), ctx():
            out = self.fn(*static)
        outs, build = _flat(out)
        if len(self._graphs) >= self.max_graphs:
            self._graphs.pop(next(iter(self._graphs)))
        self._graphs[key] = (g, static, outs, build)
        self.captures += 1
        return self._graphs[key]

    def __call__(self, *args):
        if not args or not all(isinstance(a, torch.Tensor) and a.is_cuda for a in args):
            raise TypeError("GraphedCallable: every argument must be a GPU tensor")
        key = tuple((tuple(a.shape), a.dtype, a.device) for a in args)
        if key in self._eager:
            return self._eager_call(args)
        ent = self._graphs.get(key)
        if ent is None:
            try:
                ent = self._capture(key, args)
            except Exception as e:  # noqa: BLE001 - e.g. a host sync inside fn: run it eagerly
                log.warning("HIP graph capture failed (%s: %s); running eagerly for this input shape",
                            type(e).__name__, str(e)[:200])
                torch.cuda.synchronize(args[0].device)
                self._eager.add(key)
                return self._eager_call(args)
        g, static, outs, build = ent
        for s, a in zip(static, args):
            s.copy_(a)
        g.replay()
        self.replays += 1
        return build(outs)


class GraphedModule:
    """A module whose calls replay HIP graphs (:class:`GraphedCallable` over ``module.__call__``)
    and whose every other attribute is the module's: hand it to code that only calls the model
    (an evaluation function).  On the CPU it is the module itself."""

    def __init__(self, module, **kw):
        object.__setattr__(self, "_module", module)
        object.__setattr__(self, "_graphed", GraphedCallable(module, **kw))

    def __call__(self, *args):
        if args and all(isinstance(a, torch.Tensor) and a.is_cuda for a in args):
            return self._graphed(*args)
        return self._module(*args)

    def __getattr__(self, name):
        return getattr(self._module, name)


def graphed(module, enabled: bool = True, **kw):
    """``module`` wrapped in :class:`GraphedModule` when enabled and on a GPU, else itself."""
    dev = next((p.device for p in module.parameters()), torch.device("cpu"))
    return GraphedModule(module, **kw) if enabled and dev.type == "cuda" else module
