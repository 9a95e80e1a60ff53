"""Flat parameter / gradient storage.

Every trainable parameter of a model is re-homed as a view into ONE contiguous
buffer per group (weight-decay / no-decay), and its ``.grad`` is preset to a
view of a matching flat gradient buffer.  Consequences that the rest of the
framework is built on:

* the optimizer is one kernel launch per group over billions of elements
  (``csrc/kernels/optim.hip``);
* DDP buckets are plain contiguous slices of the gradient buffer, so an
  all-reduce needs no pack/unpack copy (SURVEY.md §2.7 K5 becomes a no-op);
* an in-memory checkpoint of the whole model+optimizer state is a handful of
  large contiguous D2H copies (``easydl_amd/ckpt``);
* state transfer to a joining rank is a few large broadcasts.

A group is split at parameter boundaries into parts of at most
``EDL_FLAT_GROUP_MAX_MB`` (default 1900 MiB) of gradient bytes ("decay",
"decay.1", ...): each part is a separate allocation, so the xGMI engine can
IPC-map every gradient buffer of a multi-GB model and all-reduce its buckets in
place (segments of >= 2 GiB do not map on this platform).

Parameters are laid out in *reverse registration order* so gradients, which
backward produces roughly last-layer-first, fill buckets front to back.  Each
parameter starts on a 64-element boundary (128 B for bf16) so every view is
16-byte aligned for the vectorised kernels.
"""
from __future__ import annotations

import contextlib

import os
import weakref
from dataclasses import dataclass, field

import torch

from easydl_amd.ops import gradsink
from easydl_amd.utils import vram

ALIGN = 64


def _roundup(n: int, a: int = ALIGN) -> int:
    return (n + a - 1) // a * a


@dataclass
class ParamSlot:
    name: str
    param: torch.nn.Parameter
    offset: int
    numel: int
    shape: tuple


@dataclass
class FlatGroup:
    name: str
    weight_decay: float
    data: torch.Tensor  # model dtype (bf16 or fp32)
    grad: torch.Tensor  # grad dtype
    slots: list[ParamSlot] = field(default_factory=list)

    @property
    def numel(self) -> int:
        return self.data.numel()


def _split_by_bytes(plist, elem_bytes: int, max_bytes: int) -> list[list]:
    """Split a group's (name, param) list at parameter boundaries so that each part's
    gradient buffer stays under ``max_bytes``.  Each part is its own allocation (its own
    caching-allocator segment), so the xGMI engine can map every gradient group of a
    multi-GB model in place: IPC mappings of >= 2 GiB segments never open on this
    platform (parallel/xgmi.py REGISTER_MAX)."""
    if max_bytes <= 0:
        return [plist]
    parts, cur, used = [], [], 0
    for n, p in plist:
        b = _roundup(p.numel()) * elem_bytes
        if cur and used + b > max_bytes:
            parts.append(cur)
            cur, used = [], 0
        cur.append((n, p))
        used += b
    if cur:
        parts.append(cur)
    return parts


def await_update(p: torch.Tensor) -> None:
    """The caller's stream is about to read parameter ``p``: order it after the pending update of
    p's group on the optimizer stream, if any (ElasticTrainer._opt_overlap)."""
    ev = getattr(p, "_edl_fwd_wait", None)
    if ev is not None:
        p._edl_fwd_wait = None
        torch.cuda.current_stream(p.device).wait_event(ev)


def install_update_waits(model: torch.nn.Module) -> int:
    """Forward pre-hooks that make each module wait for the updates of the parameters it reads
    (await_update): every submodule waits for its whole subtree's parameters -- the first hook to
    run consumes the waits -- and the root for its own direct parameters, unless the model
    awaits those itself where it reads them (``model._edl_awaits_own = True``; Llama's embedding
    at the start and its head at the end).  Returns the number of hooks."""
    n = 0
    for name, mod in model.named_modules():
        root = name == ""
        if root and getattr(model, "_edl_awaits_own", False):
            continue
        params = list(mod.parameters(recurse=not root))
        if not params:
            continue

        def hook(_m, _inp, params=params):
            for p in params:
                await_update(p)
        mod.register_forward_pre_hook(hook)
        n += 1
    return n


def _pre_accumulate_hook(ref, key):
    def hook(g):
        me = ref()
        if g is not None and me is not None:   # None: a fused op delivered this gradient itself
            me.saw_autograd = True
            me._autograd_slots.add(key)
            gradsink.await_shadow(me._slot_of[key][1].param)   # AccumulateGrad writes it next
        return None
    return hook


def _post_accumulate_hook(ref):
    def hook(p):
        me = ref()
        if me is not None:
            me._post_accumulate(p)
    return hook


class FlatParams:
    """Re-home a module's parameters into flat buffers.

    Args:
        module: the model (already on its target device and dtype).
        grad_dtype: dtype of the gradient buffers (default: parameter dtype).
        no_decay: predicate ``(name, param) -> bool`` selecting the no-decay group
            (default: 1-D parameters, i.e. norms and biases).
    """

    def __init__(self, module: torch.nn.Module, weight_decay: float = 0.0, grad_dtype: torch.dtype | None = None,
                 no_decay=None, max_group_bytes: int | None = None):
        if max_group_bytes is None:
            # VRAM hand-over to a hot standby (utils/vram.py) maps every state tensor over IPC, which
            # takes allocations below 2 GiB: the fp32 master / moments of a group are 2x its bf16 size
            default_mb = vram.GROUP_MAX_MB if vram.enabled() else 1900
            max_group_bytes = int(float(os.environ.get("EDL_FLAT_GROUP_MAX_MB", default_mb)) * 2**20)
        if no_decay is None:
            no_decay = lambda n, p: p.ndim < 2  # noqa: E731
        named = [(n, p) for n, p in module.named_parameters() if p.requires_grad]
        if not named:
            raise ValueError("module has no trainable parameters")
        named.reverse()
        devices = {p.device for _, p in named}
        if len(devices) != 1:
            raise ValueError(f"FlatParams needs one device, got {devices}")
        self.device = devices.pop()
        by_dt: dict[torch.dtype, int] = {}
        for _, p in named:
            by_dt[p.dtype] = by_dt.get(p.dtype, 0) + p.numel()
        self.dtype = max(by_dt, key=by_dt.get)  # dominant parameter dtype (by elements)
        self.grad_dtype = grad_dtype or self.dtype
        # one flat group per (decay class, dtype): e.g. bf16 convs + fp32 BatchNorm in ResNet
        buckets: dict[tuple[str, torch.dtype], list] = {}
        for n, p in named:
            key = ("no_decay" if no_decay(n, p) else "decay", p.dtype)
            buckets.setdefault(key, []).append((n, p))
        self.groups: list[FlatGroup] = []
        # init values of parameters whose storage was adopted from a dead worker (utils/vram.py):
        # kept until the trainer knows where this process's state comes from (reinit_adopted)
        self._init_copies: list[tuple[torch.Tensor, torch.Tensor]] = []
        chunks = []
        for (cls, dt), plist in sorted(buckets.items(), key=lambda kv: (kv[0][0], str(kv[0][1]))):
            base = cls if dt == self.dtype else f"{cls}_{str(dt).split('.')[-1]}"
            gdt = grad_dtype if (grad_dtype is not None and dt == self.dtype) else dt
            for i, part in enumerate(_split_by_bytes(plist, torch.empty((), dtype=gdt).element_size(),
                                                     max_group_bytes)):
                chunks.append((cls, dt, gdt, base if i == 0 else f"{base}.{i}", part))
        for cls, dt, gdt, gname, plist in chunks:
            total = sum(_roundup(p.numel()) for _, p in plist)
            data = vram.take(f"flat/{gname}/data", total, dt, self.device, keep=True)
            grad = vram.take(f"flat/{gname}/grad", total, gdt, self.device)
            adopted = data is not None   # the previous worker's weights: not overwritten by this init
            data = torch.zeros(total, dtype=dt, device=self.device) if data is None else data
            grad = torch.zeros(total, dtype=gdt, device=self.device) if grad is None else grad
            grp = FlatGroup(gname, weight_decay if cls == "decay" else 0.0, data, grad)
            off = 0
            for n, p in plist:
                k = p.numel()
                view = data[off:off + k].view(p.shape)
                if not adopted:
                    with torch.no_grad():
                        view.copy_(p.data)
                else:
                    self._init_copies.append((view, p.data))
                p.data = view
                if gdt != dt and hasattr(p, "grad_dtype"):
                    # fp32 gradient buffers under bf16 parameters (grad_dtype=fp32): torch >= 2.10
                    # checks .grad against the tensor's grad_dtype; autograd-path gradients are
                    # then accumulated into the fp32 buffer
                    p.grad_dtype = gdt
                p.grad = grad[off:off + k].view(p.shape)
                p._edl_flat = True
                p._edl_fresh = True
                p._edl_name = n
                grp.slots.append(ParamSlot(n, p, off, k, tuple(p.shape)))
                off += _roundup(k)
            self.groups.append(grp)
        self.saw_autograd = False
        self._autograd_slots: set = set()   # (group, slot) that autograd accumulated into
        self._slot_of = {id(s.param): (g, s) for g in self.groups for s in g.slots}
        # autograd-path parameters (ops that return the gradient) accumulate in place.  A
        # fused op that delivers its gradient directly returns None, and the post-accumulate
        # hook still fires for it; only the tensor hook sees whether a gradient really
        # reached AccumulateGrad, so that is what marks a slot for zeroing.
        # The hooks reach this object through a weak reference: a tensor hook lives in the
        # parameter's C++ autograd metadata, which Python's cycle collector cannot traverse, so
        # parameter -> hook -> FlatParams -> parameter was a cycle that was never collected (a
        # standby's warm-up model and its flat buffers stayed allocated: ~7 B/param per warm-up,
        # profiles/r05_ttr_headline.md, "What changed" item 3).
        me = weakref.ref(self)
        for g in self.groups:
            for s in g.slots:
                s.param.register_hook(_pre_accumulate_hook(me, id(s.param)))
                s.param.register_post_accumulate_grad_hook(_post_accumulate_hook(me))
        self._ready_cb = None
        self.gshadow: list[torch.Tensor] | None = None      # ensure_shadow
        self.gshadow_loss: torch.Tensor | None = None
        if vram.pending(f"flat/{self.groups[0].name}/gshadow"):
            self.ensure_shadow()    # a dead worker's shadow: taken now, before unused adoptions are dropped

    # -- gradient shadow ------------------------------------------------------
    def ensure_shadow(self, pool=None) -> None:
        """A second copy of every gradient buffer, plus the partial loss: the trainer copies the
        accumulated gradients into it after each micro-batch but the last (ElasticTrainer
        _shadow_grads, step marks ``gstep`` / ``gmb``).  A replacement that adopts the dead
        worker's HBM then resumes the interrupted step at its first unfinished micro-batch
        instead of recomputing the whole step.  Bytes: one gradient buffer (16 GB for
        Llama-3-8B with bf16 gradients), affordable in 288 GB of HBM."""
        if self.gshadow is not None:
            return
        sh = []
        # ``pool`` (a torch.cuda.MemPool): allocated after training started, a buffer must not be
        # carved out of a cached activation segment -- its IPC export would map that whole segment
        ctx = torch.cuda.use_mem_pool(pool) if pool is not None else contextlib.nullcontext()
        with ctx:
            for g in self.groups:
                t = vram.take(f"flat/{g.name}/gshadow", g.grad.numel(), g.grad.dtype, self.device, keep=True)
                sh.append(torch.empty_like(g.grad) if t is None else t)
            loss = vram.take("flat/gshadow_loss", 1, torch.float32, self.device, keep=True)
            self.gshadow_loss = torch.zeros(1, dtype=torch.float32, device=self.device) if loss is None else loss
        self.gshadow = sh

    def shadow_tensors(self) -> dict[str, torch.Tensor]:
        if self.gshadow is None:
            return {}
        ts = {f"flat/{g.name}/gshadow": t for g, t in zip(self.groups, self.gshadow)}
        ts["flat/gshadow_loss"] = self.gshadow_loss
        return ts

    def load_shadow(self) -> None:
        """Gradients := the shadow (a mid-step resume); every parameter then accumulates."""
        with torch.no_grad():
            for g, t in zip(self.groups, self.gshadow):
                g.grad.copy_(t)
        self.mark_accumulating()

    def mark_accumulating(self) -> None:
        """The gradient buffers hold a partial sum: every later write accumulates onto it."""
        for g in self.groups:
            for s in g.slots:
                s.param._edl_fresh = False

    # -- gradient protocol -------------------------------------------------
    def _post_accumulate(self, p):
        p._edl_fresh = False
        if self._ready_cb is not None:
            self._ready_cb(p)

    def set_ready_callback(self, cb) -> None:
        """``cb(param)`` fires when a parameter's gradient is complete for this backward."""
        self._ready_cb = cb
        for g in self.groups:
            for s in g.slots:
                s.param._edl_ready_cb = cb

    def zero_grad(self) -> None:
        """Start a new accumulation window.

        Direct-writing ops overwrite on their first write, so no memset is
        needed unless an autograd-path parameter accumulated last time.  Also
        starts a new weight generation: parameters may have changed since the
        last step, so cached transposed weight copies are refreshed on use.
        """
        from easydl_amd.ops.fused import new_weight_generation
        new_weight_generation()
        if self.saw_autograd:
            # only the slots autograd accumulated into (direct writers overwrite anyway):
            # ResNet-50 / Llama no longer memset their whole gradient buffer every step
            if len(self._autograd_slots) * 4 > sum(len(g.slots) for g in self.groups):
                for g in self.groups:
                    for s in g.slots:
                        gradsink.await_shadow(s.param)   # (an optimizer still reading them)
                    g.grad.zero_()
            else:
                for key in self._autograd_slots:
                    g, s = self._slot_of[key]
                    gradsink.await_shadow(s.param)
                    g.grad[s.offset:s.offset + s.numel].zero_()
            self.saw_autograd = False
            self._autograd_slots = set()
        for g in self.groups:
            for s in g.slots:
                s.param._edl_fresh = True
                # autograd may have replaced .grad (e.g. set_to_none elsewhere): re-bind
                if s.param.grad is None or s.param.grad.data_ptr() != g.grad[s.offset:].data_ptr():
                    s.param.grad = g.grad[s.offset:s.offset + s.numel].view(s.shape)

    def finalize_untouched(self) -> None:
        """Zero gradients of parameters that received none this window (unused params)."""
        for g in self.groups:
            for s in g.slots:
                if gradsink.is_fresh(s.param):
                    s.param.grad.zero_()
                    s.param._edl_fresh = False

    # -- adopted storage ------------------------------------------------------
    def reinit_adopted(self) -> int:
        """Adopted weights that nothing will overwrite (no HBM resume, no snapshot, no state
        transfer): back to this process's own seeded init values, as a fresh start would have
        them.  Returns the number of parameters re-initialised."""
        with torch.no_grad():
            for view, init in self._init_copies:
                view.copy_(init)
        n = len(self._init_copies)
        self._init_copies = []
        return n

    def drop_init_copies(self) -> None:
        """The state is settled (resumed, restored or transferred): free the init values."""
        self._init_copies = []

    def rehome(self, adopted, can_continue=lambda: True) -> int:
        """Move every buffer ``adopted(tensor)`` says is built on adopted memory (a dead worker's
        HBM, mapped over IPC) into this process's own allocation -- same values, parameters and gradients re-pointed --
        one group at a time, so the extra memory is one group.  A process cannot export memory
        it imported, so only re-homed state can be handed to the next standby.  Stops before a
        group when ``can_continue()`` is False.  Returns the number of buffers moved."""
        n = 0
        with torch.no_grad():
            for g in self.groups:
                if not can_continue():
                    break
                if adopted(g.data):
                    new = torch.empty_like(g.data)
                    new.copy_(g.data)
                    for s in g.slots:
                        s.param.data = new[s.offset:s.offset + s.numel].view(s.shape)
                    g.data = new
                    n += 1
                if adopted(g.grad):
                    new = torch.empty_like(g.grad)
                    new.copy_(g.grad)
                    for s in g.slots:
                        s.param.grad = new[s.offset:s.offset + s.numel].view(s.shape)
                    g.grad = new
                    n += 1
            for i, t in enumerate(self.gshadow or []):
                if adopted(t) and can_continue():
                    self.gshadow[i] = t.clone()
                    n += 1
            if self.gshadow_loss is not None and adopted(self.gshadow_loss):
                self.gshadow_loss = self.gshadow_loss.clone()
                n += 1
        return n

    # -- views ---------------------------------------------------------------
    def params(self):
        for g in self.groups:
            for s in g.slots:
                yield s.param

    def named_slots(self):
        for g in self.groups:
            for s in g.slots:
                yield g, s

    @property
    def numel(self) -> int:
        return sum(g.numel for g in self.groups)

    def num_params(self) -> int:
        return sum(s.numel for _, s in self.named_slots())


class FlatBuffers:
    """Persistent module buffers (BatchNorm running statistics and batch counters)
    re-homed into one flat tensor per dtype, the way :class:`FlatParams` does for
    parameters.  The trainer adds these tensors to the training state, so they
    reach joiners in the state broadcast and go into in-memory snapshots and
    persisted checkpoints.  The reference leaves the checkpoint contents undefined
    (SURVEY.md §5.4); without this a replacement worker would restart its running
    statistics from their initial values.  Non-persistent buffers (derived tables)
    stay where they are."""

    def __init__(self, module: torch.nn.Module):
        by_dtype: dict[torch.dtype, list] = {}
        seen = set()
        for mod in module.modules():
            skip = getattr(mod, "_non_persistent_buffers_set", set())
            for name, b in mod._buffers.items():
                if b is None or name in skip:
                    continue
                if id(b) in seen:
                    raise ValueError(f"buffer {name} is registered by more than one module")
                seen.add(id(b))
                by_dtype.setdefault(b.dtype, []).append((mod, name, b))
        self.tensors: dict[str, torch.Tensor] = {}
        self._init_copies: list[tuple[torch.Tensor, torch.Tensor]] = []
        self._where: dict[str, list] = {}   # dtype key -> (module, buffer name, offset, shape)
        for dt, items in by_dtype.items():
            key = str(dt).replace("torch.", "")
            n = sum(b.numel() for _, _, b in items)
            dev = items[0][2].device
            # a dead worker's running statistics (utils/vram.py), kept for an HBM resume
            flat = vram.take(f"bufs/{key}", n, dt, dev, keep=True)
            adopted = flat is not None
            flat = torch.empty(n, dtype=dt, device=dev) if flat is None else flat
            off = 0
            with torch.no_grad():
                for mod, name, b in items:
                    view = flat[off:off + b.numel()].view(b.shape)
                    if adopted:
                        self._init_copies.append((view, b))
                    else:
                        view.copy_(b)
                    mod._buffers[name] = view
                    self._where.setdefault(key, []).append((mod, name, off, tuple(b.shape)))
                    off += b.numel()
            self.tensors[key] = flat

    def reinit_adopted(self) -> int:
        """See :meth:`FlatParams.reinit_adopted`."""
        with torch.no_grad():
            for view, init in self._init_copies:
                view.copy_(init)
        n = len(self._init_copies)
        self._init_copies = []
        return n

    def drop_init_copies(self) -> None:
        self._init_copies = []

    def rehome(self, adopted, can_continue=lambda: True) -> int:
        """See :meth:`FlatParams.rehome`."""
        n = 0
        with torch.no_grad():
            for key, flat in list(self.tensors.items()):
                if not adopted(flat) or not can_continue():
                    continue
                new = flat.clone()
                for mod, name, off, shape in self._where.get(key, []):
                    numel = 1
                    for d in shape:
                        numel *= d
                    mod._buffers[name] = new[off:off + numel].view(shape)
                self.tensors[key] = new
                n += 1
        return n
