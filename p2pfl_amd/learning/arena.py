"""Flat parameter arenas.

MI355X-first replacement for the reference's per-layer ``state_dict`` handling
(``lightning_learner.py:113-164``, ``fedavg.py:49-58``): a model's parameters
and buffers live in ONE contiguous fp32 device buffer, and every named tensor
is a view into it.  Aggregation, optimizer steps, gossip snapshots and wire
(de)serialisation then operate on a single buffer -- one kernel launch or one
copy instead of one per layer.

* :class:`ParamLayout` -- names, shapes, original dtypes and 64-element
  (256-byte) aligned offsets; identical across peers running the same model.
* :class:`FlatParams`  -- an ``OrderedDict`` of views that also carries
  ``.flat`` (the 1-D buffer) and ``.layout``; it is what ``get_parameters``
  returns, so ``params[name]`` indexing keeps working
  (reference ``utils.py:129-137``).
* :func:`bind_module` -- re-homes an ``nn.Module``'s parameters/buffers (and
  optionally their gradients) into arenas, so the live model *is* the arena.
"""

from __future__ import annotations

from collections import OrderedDict
from dataclasses import dataclass
from typing import Any, Dict, Iterable, Mapping, Optional, Tuple

import torch

ALIGN = 64  # elements (256 B of fp32): keeps every view 16-B aligned for dwordx4 access


def _align(n: int) -> int:
    return (n + ALIGN - 1) // ALIGN * ALIGN


@dataclass(frozen=True)
class ParamLayout:
    names: Tuple[str, ...]
    shapes: Tuple[Tuple[int, ...], ...]
    dtypes: Tuple[str, ...]
    offsets: Tuple[int, ...]
    numel: int  # padded total length of the flat buffer

    @classmethod
    def from_tensors(cls, items: Iterable[Tuple[str, torch.Tensor]]) -> "ParamLayout":
        names, shapes, dtypes, offsets = [], [], [], []
        off = 0
        for name, t in items:
            names.append(name)
            shapes.append(tuple(int(s) for s in t.shape))
            dtypes.append(str(t.dtype).replace("torch.", ""))
            offsets.append(off)
            off = _align(off + t.numel())
        return cls(tuple(names), tuple(shapes), tuple(dtypes), tuple(offsets), max(off, ALIGN))

    def sizes(self) -> Tuple[int, ...]:
        out = []
        for s in self.shapes:
            n = 1
            for d in s:
                n *= d
            out.append(n)
        return tuple(out)

    def compatible(self, other: "ParamLayout") -> bool:
        return self.shapes == other.shapes and self.offsets == other.offsets and self.numel == other.numel

    def to_json(self) -> Dict:
        return {
            "names": list(self.names),
            "shapes": [list(s) for s in self.shapes],
            "dtypes": list(self.dtypes),
            "offsets": list(self.offsets),
            "numel": self.numel,
        }

    @classmethod
    def from_json(cls, d: Dict) -> "ParamLayout":
        return cls(
            tuple(d["names"]),
            tuple(tuple(int(x) for x in s) for s in d["shapes"]),
            tuple(d["dtypes"]),
            tuple(int(o) for o in d["offsets"]),
            int(d["numel"]),
        )


class FlatParams(OrderedDict):
    """Named views into one contiguous fp32 buffer."""

    flat: torch.Tensor
    layout: ParamLayout

    @classmethod
    def from_flat(cls, flat: torch.Tensor, layout: ParamLayout) -> "FlatParams":
        if flat.dim() != 1 or flat.numel() < layout.numel or not flat.is_contiguous():
            raise ValueError("flat buffer does not match layout")
        out = cls()
        for name, shape, off, n in zip(layout.names, layout.shapes, layout.offsets, layout.sizes()):
            out[name] = flat[off : off + n].view(shape)
        out.flat = flat
        out.layout = layout
        return out

    @property
    def nbytes(self) -> int:
        return self.flat.numel() * self.flat.element_size()

    @property
    def device(self) -> torch.device:
        return self.flat.device

    def clone(self) -> "FlatParams":  # type: ignore[override]
        with reading(self):  # a learner's live weights: after its last write (WeightGuard)
            return FlatParams.from_flat(self.flat.clone(), self.layout)

    def to(self, device: torch.device, non_blocking: bool = False) -> "FlatParams":
        if self.flat.device == torch.device(device):
            return self
        with reading(self):
            return FlatParams.from_flat(self.flat.to(device, non_blocking=non_blocking), self.layout)


class WeightGuard:
    """Lazy stream ordering of one learner's live weights (the arena) across HIP streams.

    The learner writes its weights on its own compute stream (``fit``,
    ``set_parameters``); other threads read them on theirs (the FedAvg fold, the
    gossip snapshot, wire encoding, checkpoints).  Instead of handing the whole
    compute stream back to the caller's stream after every block -- a cross-queue
    wait that cost the next epoch ~0.55 ms of device time per round
    (``profiles/r5_handoff_probe.md``) -- each write block records a ready event,
    and each reader waits on it only where it launches a read (RAW); readers record
    an event after their reads, which the next write block waits on (WAR).  A
    block whose predecessor ran on the same stream waits on nothing: a lone
    trainer pays no hand-off at all.  Replaces the reference's synchronous
    ``learner.get_parameters()`` after ``fit`` (``train_stage.py:70-74``,
    ``lightning_learner.py:180-198``), where Lightning finished the epoch on the host.
    """

    def __init__(self) -> None:
        import threading

        self._lock = threading.Lock()
        self._ready: Optional[Tuple[Any, Any]] = None  # (event, stream) after the last write block
        self._reads: Dict[Any, Any] = {}  # stream -> event after the latest reads on it since then
        self._handed: Dict[Any, None] = {}  # streams the weights were handed to with no read event

    @staticmethod
    def _gated():
        from p2pfl_amd.learning.step_graph import GATE

        return GATE.shared()  # event record / wait on the default stream: never beside a capture

    def acquire(self, stream: Any) -> None:
        """Order work about to be launched on ``stream`` after the last write of the weights."""
        if stream is None:
            return
        with self._lock:
            r = self._ready
        if r is not None and r[1] != stream:
            with self._gated():
                stream.wait_event(r[0])

    def release(self, stream: Any) -> None:
        """Reads of the weights were launched on ``stream``: the next write waits for them."""
        if stream is None:
            return
        with self._gated():
            ev = torch.cuda.Event()
            ev.record(stream)
        with self._lock:
            self._reads[stream] = ev

    def hand_out(self, stream: Any) -> None:
        """The weights were given to code that may read them on ``stream`` without
        recording when it is done (a public ``get_parameters()``): the stream waits
        for the last write now, and the next write waits for everything queued on
        it until then."""
        if stream is None:
            return
        self.acquire(stream)
        with self._lock:
            self._handed[stream] = None

    def begin_write(self, stream: Any) -> None:
        """A write block starts on ``stream``: after every read and the previous write
        launched on other streams."""
        if stream is None:
            return
        with self._lock:
            waits = [ev for s, ev in self._reads.items() if s != stream]
            handed = [s for s in self._handed if s != stream]
            self._reads = {}
            self._handed = {}
            r = self._ready
        if r is not None and r[1] != stream:
            waits.append(r[0])
        if waits or handed:
            with self._gated():
                for ev in waits:
                    stream.wait_event(ev)
                for s in handed:
                    stream.wait_stream(s)

    def end_write(self, stream: Any) -> None:
        if stream is None:
            return
        with self._gated():
            ev = torch.cuda.Event()
            ev.record(stream)
        with self._lock:
            self._ready = (ev, stream)


class reading:
    """``with reading(params): <launch reads of params.flat on the current stream>`` --
    the :class:`WeightGuard` hand-off for a learner's live weights (a no-op for any
    other FlatParams and on the CPU)."""

    def __init__(self, params: Any) -> None:
        self.guard = getattr(params, "guard", None)
        flat = getattr(params, "flat", None)
        self.stream = torch.cuda.current_stream(flat.device) if (self.guard is not None and flat is not None and flat.is_cuda) else None

    def __enter__(self) -> "reading":
        if self.stream is not None:
            self.guard.acquire(self.stream)
        return self

    def __exit__(self, *exc) -> None:
        if self.stream is not None:
            self.guard.release(self.stream)


def flatten(params: Mapping[str, torch.Tensor], device: Optional[torch.device] = None) -> FlatParams:
    """Return ``params`` as a :class:`FlatParams` (no copy if it already is one)."""
    if isinstance(params, FlatParams) and (device is None or params.flat.device == torch.device(device)):
        return params
    items = list(params.items())
    layout = ParamLayout.from_tensors(items)
    if device is None:
        device = items[0][1].device if items else torch.device("cpu")
    flat = torch.zeros(layout.numel, dtype=torch.float32, device=device)
    for (name, t), off in zip(items, layout.offsets):
        flat[off : off + t.numel()].copy_(t.detach().reshape(-1), non_blocking=True)
    return FlatParams.from_flat(flat, layout)


def is_arena_view(t: torch.Tensor, flat: torch.Tensor) -> bool:
    base = flat.data_ptr()
    return flat.device == t.device and base <= t.data_ptr() < base + flat.numel() * flat.element_size()


class ModuleArena:
    """Binds an ``nn.Module``'s state into flat arenas.

    After binding, every float parameter and buffer of the module is a view of
    ``self.params.flat``; with ``grads=True`` each parameter's ``.grad`` is a
    view of ``self.grads`` (so a single fused optimizer kernel can update the
    whole model).  Integer buffers (e.g. BatchNorm's ``num_batches_tracked``)
    stay where they are but are mirrored into the arena by :meth:`sync_in`
    and restored by :meth:`sync_out`.
    """

    def __init__(
        self,
        module: torch.nn.Module,
        device: Optional[torch.device] = None,
        grads: bool = False,
        compute_dtype: Optional[torch.dtype] = None,
        fp32_names: Optional[Iterable[str]] = None,
        channels_last_names: Optional[Iterable[str]] = None,
    ) -> None:
        sd = module.state_dict(keep_vars=True)
        if device is None:
            device = next(iter(sd.values())).device if sd else torch.device("cpu")
        self.module = module
        self.layout = ParamLayout.from_tensors((k, v) for k, v in sd.items())
        flat = torch.zeros(self.layout.numel, dtype=torch.float32, device=device)
        self.params = FlatParams.from_flat(flat, self.layout)
        self.params.guard = WeightGuard()  # stream ordering of the live weights (learner hand-offs)
        self._int_buffers: Dict[str, torch.Tensor] = {}
        for name, t in sd.items():
            view = self.params[name]
            view.copy_(t.detach().reshape(view.shape).to(device=device, dtype=torch.float32))
            if t.is_floating_point():
                t.data = view  # parameter / buffer now lives in the arena
            else:
                self._int_buffers[name] = t
        self.grads: Optional[torch.Tensor] = None
        if grads:
            self.grads = torch.zeros_like(flat)
            gviews = FlatParams.from_flat(self.grads, self.layout)
            for name, p in module.named_parameters():
                if name in gviews:
                    p.grad = gviews[name]
        # mask of trainable elements (params, not buffers)
        self.param_names = [n for n, _ in module.named_parameters()]
        # Mixed precision (GPU learners): the module's matrix weights become
        # bf16 views of a shadow arena that the optimizer rewrites after every
        # step, so GEMMs/convs read bf16 weights directly -- no autocast cast
        # kernel per weight per forward, no cast-back kernel per gradient.
        # The fp32 arena stays the master copy (FedAvg, gossip, checkpoints).
        self.shadow: Optional[torch.Tensor] = None
        self.shadow_names: Tuple[str, ...] = ()
        self.shadow_cl: Dict[str, Tuple[int, Tuple[int, ...]]] = {}
        if compute_dtype is not None:
            if grads:
                raise ValueError("mixed-precision arenas keep per-tensor grads (grads=False)")
            keep = set(fp32_names) if fp32_names is not None else {n for n, p in module.named_parameters() if p.dim() < 2}
            # Conv weights named in ``channels_last_names`` get a channels-last
            # (O, kh, kw, I) shadow region: with NHWC activations MIOpen then
            # reads the weight as is and returns its gradient in the same
            # layout, instead of a relayout copy of every conv weight per
            # forward/backward and of every weight gradient per step.  The
            # fp32 master (wire, FedAvg, checkpoints) keeps the OIHW order;
            # the multi-tensor optimizer maps between the two.
            cl = set(channels_last_names or ())
            self.shadow = torch.empty(self.layout.numel, dtype=compute_dtype, device=device)
            names = []
            for name, p in module.named_parameters():
                if name in keep:
                    continue
                off = self.layout.offsets[self.layout.names.index(name)]
                region = self.shadow[off : off + p.numel()]
                if name in cl and p.dim() == 4 and p.shape[2] * p.shape[3] > 1:
                    o, i, kh, kw = p.shape
                    self.shadow_cl[name] = (off, tuple(p.shape))
                    p.data = region.view(o, kh, kw, i).permute(0, 3, 1, 2)
                else:
                    p.data = region.view(p.shape)
                names.append(name)
            self.shadow_names = tuple(names)
            self.refresh_shadow()

    @property
    def flat(self) -> torch.Tensor:
        return self.params.flat

    def refresh_shadow(self) -> None:
        """Rewrite the compute-dtype shadow from the fp32 master (channels-last regions permuted)."""
        if self.shadow is None:
            return
        flat = self.params.flat
        self.shadow.copy_(flat)
        for off, (o, i, kh, kw) in self.shadow_cl.values():
            n = o * i * kh * kw
            self.shadow[off : off + n].view(o, kh, kw, i).copy_(flat[off : off + n].view(o, i, kh, kw).permute(0, 2, 3, 1))

    def sync_in(self) -> None:
        """Mirror non-float buffers into the arena (before sending / aggregating)."""
        for name, t in self._int_buffers.items():
            self.params[name].copy_(t.reshape(self.params[name].shape).float())

    def sync_out(self) -> None:
        """Copy averaged non-float buffers back to the module; refresh the bf16 shadow."""
        for name, t in self._int_buffers.items():
            t.copy_(self.params[name].reshape(t.shape).round().to(t.dtype))
        if self.shadow is not None:
            self.refresh_shadow()

    def grads_bound(self) -> bool:
        if self.grads is None:
            return False
        for _, p in self.module.named_parameters():
            if p.grad is None or not is_arena_view(p.grad, self.grads):
                return False
        return True

    def rebind_grads(self) -> None:
        if self.grads is None:
            return
        gviews = FlatParams.from_flat(self.grads, self.layout)
        for name, p in self.module.named_parameters():
            if p.grad is not None and not is_arena_view(p.grad, self.grads):
                gviews[name].copy_(p.grad)
            p.grad = gviews[name]
