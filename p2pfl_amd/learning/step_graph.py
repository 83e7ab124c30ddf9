"""One training step captured as a HIP graph (mixed-precision torch learners).

A ResNet / ViT training step on PyTorch-ROCm is a few hundred kernel launches
(convolutions / GEMMs, the fused BatchNorm or LayerNorm kernels, autograd's
bookkeeping, the multi-tensor optimizer).  At the federated batch size (32)
most of them run for a few microseconds, so the step is bound by host-side
launch work, not by the GPU.  :class:`TrainStepGraph` records the whole step
ONCE -- batch gather from the device-resident shard, forward under bf16
autocast, backward, fused optimizer -- and then replays it with a single
``hipGraphLaunch`` per step.  Only the batch's sample indices change between
replays (one 256-byte device copy into the graph's static index buffer).

Semantics are those of the eager loop: same batches in the same order, the
same optimizer math (the optimizer's step count and bias corrections live on
the device, see :class:`~p2pfl_amd.learning.optim.MTAdam`), BatchNorm running
statistics updated inside the graph.  The first step of every ``fit`` (which
seeds SGD momentum) and a short last batch run eagerly.
"""

from __future__ import annotations

import gc
import threading
from contextlib import contextmanager
from typing import Any, Optional, Tuple

import torch

from p2pfl_amd.data.datamodule import wants_float
from p2pfl_amd.ops.fused import deferred_param_grads

from p2pfl_amd.ops import splitk
from p2pfl_amd.utils.lockcheck import make_lock
from p2pfl_amd.utils.streams import private_stream

# virtual peers (one node thread each) may capture concurrently: serialise
# captures process-wide.  Captures run in "relaxed" error mode: the exclusive
# device gate already keeps every other learner's GPU work out of the recording
# window, and what other threads may still do then -- drop the last reference to
# a graph / event (a destroy call), wait on an event in a completion thread --
# must not invalidate this thread's capture (in "thread_local" mode on ROCm it
# did: the process aborted in tests/test_gpu_node.py::test_virtual_peers_on_gpu).
_CAPTURE_LOCK = make_lock("StepGraph._CAPTURE_LOCK")


class DeviceGate:
    """Shared/exclusive gate of the GPU work of the learners of one process.

    Virtual peers train concurrently, one node thread each.  A HIP-graph
    capture must not overlap another peer's eager work (its autograd
    backward runs on the engine's shared device thread, its library calls
    may synchronise), so every learner step runs under ``shared()`` and every
    capture under ``exclusive()``; neither is ever taken while holding the
    other, so the gate cannot deadlock.
    """

    def __init__(self) -> None:
        self._cv = threading.Condition()
        self._shared = 0
        self._excl = False
        self._owner: Optional[int] = None  # thread holding the gate exclusively

    @contextmanager
    def shared(self):
        if self._owner == threading.get_ident():  # the exclusive holder already has the device
            yield
            return
        with self._cv:
            while self._excl:
                self._cv.wait()
            self._shared += 1
        try:
            yield
        finally:
            with self._cv:
                self._shared -= 1
                self._cv.notify_all()

    @contextmanager
    def exclusive(self):
        with self._cv:
            while self._excl or self._shared:
                self._cv.wait()
            self._excl = True
            self._owner = threading.get_ident()
        try:
            yield
        finally:
            with self._cv:
                self._excl = False
                self._owner = None
                self._cv.notify_all()


GATE = DeviceGate()

# First warm-ups per model structure: the first peer of a process to warm up a
# given step runs it with the device to itself -- its per-shape autotune timings
# (ops/autotune.py, cached process-wide) then see no other peer's kernels, and
# the other peers' warm-ups, which follow under the shared gate, find every
# choice made (the round-4 overlap run: eight peers timing and capturing at
# once made the first round 2.4x longer).
_WARMED: set = set()
_WARM_LOCK = threading.Lock()


@contextmanager
def warmup_gate(key: Tuple):
    """Exclusive gate for the first warm-up of ``key`` in this process, shared after."""
    with _WARM_LOCK:
        first = key not in _WARMED
    if not first:
        with GATE.shared():
            yield
        return
    with GATE.exclusive():
        yield
    with _WARM_LOCK:
        _WARMED.add(key)


@contextmanager
def no_gc(collect: bool = True):
    """Collect now (unless the caller just did, outside its locks), then keep
    Python's cyclic GC off for the capture: a collection during capture can run
    the destructor of an unrelated object holding device resources (another
    learner's graph, events, streams) -- a HIP call that invalidates this
    thread's capture and aborts the process."""
    if collect:
        gc.collect()
    was = gc.isenabled()
    gc.disable()
    try:
        yield
    finally:
        if was:
            gc.enable()


def graphable_loader(loader: Any) -> bool:
    return all(hasattr(loader, a) for a in ("x", "y", "permutation", "normalize", "batch_size")) and loader.x.is_cuda


class TrainStepGraph:
    """HIP graph of one training step of ``batch`` samples (default the loader's
    batch; the learner captures a second one for an epoch's short last batch)."""

    def __init__(self, learner: Any, opt: Any, loader: Any, batch: Optional[int] = None) -> None:
        self.learner = learner
        self.opt = opt
        self.loader = loader
        self.B = int(batch or loader.batch_size)
        dev = learner.device
        self.key = self.make_key(learner, opt, loader, self.B)
        self.idx = torch.zeros(self.B, dtype=torch.int64, device=dev)
        self.gtab = torch.zeros(len(opt.mt.params), dtype=torch.int64, device=dev)
        self.stream = private_stream(dev)
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.loss: Optional[torch.Tensor] = None

    @staticmethod
    def make_key(learner: Any, opt: Any, loader: Any, batch: Optional[int] = None) -> Tuple:
        return (id(opt), opt.config(), int(batch or loader.batch_size), loader.x.data_ptr(), loader.y.data_ptr(),
                learner.arena.flat.data_ptr(), id(learner.model))

    # -- body ---------------------------------------------------------------
    def _body(self, graph: bool) -> torch.Tensor:
        ld, model, opt = self.loader, self.learner.model, self.opt
        x = ld.x.index_select(0, self.idx)
        if wants_float(ld, model):
            x = x.float().div_(255.0)
        y = ld.y.index_select(0, self.idx)
        for p in opt.mt.params:
            p.grad = None
        with deferred_param_grads():  # column-sum parameter gradients reduced in one launch at the end
            with torch.autocast(device_type="cuda", dtype=torch.bfloat16, cache_enabled=False):
                loss = model.training_step((x, y), 0)
            loss.backward()
        if graph:
            opt.step_graph(self.gtab)
        else:
            opt.step()
        model.pop_logged()
        return loss.detach()

    def capture(self, idx: torch.Tensor) -> None:
        """Warm up, then capture; parameters, optimizer and BN state are restored after the warm-up.

        The warm-up step does every lazy first use -- workspaces, the per-shape
        autotune timing (``ops/autotune.py``), library solver choices -- which
        can take seconds on a fresh device.  The first warm-up of a model
        structure in the process takes the gate exclusively (clean autotune
        timings, see :func:`warmup_gate`); later ones are ordinary eager work
        under the SHARED gate next to the other peers' steps.  The capture
        itself (host-side recording, no kernel executes) takes the gate
        exclusively, so a capturing peer stalls the others only for the
        recording (reference requirement: training must not stall the node,
        ``train_stage.py:88-93``).
        """
        learner, opt = self.learner, self.opt
        arena = learner.arena
        dev = learner.device
        cur = torch.cuda.current_stream(dev)
        wkey = ("train", type(learner.model).__name__, self.B, tuple(self.loader.x.shape[1:]), opt.config())
        with warmup_gate(wkey):
            self.stream.wait_stream(cur)
            with torch.cuda.stream(self.stream):
                keep = [t for t in [arena.flat, arena.shadow] + opt.state_tensors() if t is not None]
                saved = [t.clone() for t in keep]
                ints = {k: v.clone() for k, v in getattr(arena, "_int_buffers", {}).items()}
                t_host = opt.t
                self.idx.copy_(idx)
                self._body(graph=False)  # lazy inits (workspaces, solver choices) outside the capture
                for dst, src in zip(keep, saved):
                    dst.copy_(src)
                for k, v in ints.items():
                    arena._int_buffers[k].copy_(v)
            self.stream.synchronize()
            del saved, ints
            opt.t = t_host
            for p in opt.mt.params:  # eager gradients are not the graph's
                p.grad = None
        with GATE.shared():  # before the exclusive section (a full collection can take a while), but
            gc.collect()  # never while another thread records: a destructor's HIP call would break its capture
        with GATE.exclusive(), _CAPTURE_LOCK:
            torch.cuda.synchronize(dev)
            g = torch.cuda.CUDAGraph()
            self.counters = splitk.GraphCounters(dev)  # split-K tile counters owned by this graph
            with no_gc(collect=False), splitk.graph_scope(self.counters), torch.cuda.graph(g, stream=self.stream, capture_error_mode="relaxed"):
                self.loss = self._body(graph=True)
            opt.mt.fill_grad_table(self.gtab)  # the graph's gradient buffers, fixed for every replay
            opt.t = t_host  # recording executed nothing; host-side counters back to the pre-capture state
            for p in opt.mt.params:  # eager steps allocate their own gradients
                p.grad = None
            torch.cuda.synchronize(dev)
        self.graph = g

    def run(self, idx: torch.Tensor) -> torch.Tensor:
        """One training step on the samples ``idx`` (len == this graph's batch)."""
        self.idx.copy_(idx, non_blocking=True)
        assert self.graph is not None
        self.graph.replay()
        self.opt.t += 1
        return self.loss


class EvalStepGraph:
    """HIP graph of one evaluation step: batch gather, forward, the model's
    eval hook (loss / metric), and per-metric sums accumulated on the device.

    A pass replays it once per full batch and reads the sums back once at
    the end (one host sync per pass instead of one per logged value).
    """

    def __init__(self, learner: Any, loader: Any, hook: Any, batch: Optional[int] = None,
                 sums_of: Optional["EvalStepGraph"] = None) -> None:
        self.learner = learner
        self.loader = loader
        self.hook = hook
        self.B = int(batch or loader.batch_size)
        dev = learner.device
        self.key = self.make_key(learner, loader, hook, self.B)
        self.idx = torch.zeros(self.B, dtype=torch.int64, device=dev)
        # a pass's remainder graph accumulates into the full-batch graph's sums
        self.keys: list = list(sums_of.keys) if sums_of is not None else []
        self.sums: Optional[torch.Tensor] = sums_of.sums if sums_of is not None else None
        self.stream = private_stream(dev)
        self.graph: Optional[torch.cuda.CUDAGraph] = None

    @staticmethod
    def make_key(learner: Any, loader: Any, hook: Any, batch: Optional[int] = None) -> Tuple:
        return (getattr(hook, "__name__", str(hook)), int(batch or loader.batch_size), loader.x.data_ptr(), loader.y.data_ptr(),
                learner.arena.flat.data_ptr(), id(learner.model))

    def batch(self, idx: torch.Tensor):
        ld = self.loader
        x = ld.x.index_select(0, idx)
        if wants_float(ld, self.learner.model):
            x = x.float().div_(255.0)
        return x, ld.y.index_select(0, idx)

    def step(self, idx: torch.Tensor, weight: float, cache: bool = True) -> None:
        """Eager evaluation of one batch, accumulated into the sums (also the captured body)."""
        with torch.autocast(device_type="cuda", dtype=torch.bfloat16, cache_enabled=cache):
            self.hook(self.batch(idx), 0)
        logged = self.learner.model.pop_logged()
        if not self.keys:
            self.keys = sorted(logged)
            self.sums = torch.zeros(len(self.keys), dtype=torch.float32, device=self.learner.device)
        for j, k in enumerate(self.keys):
            v = logged[k]
            v = v.float() if isinstance(v, torch.Tensor) else torch.tensor(float(v), device=self.learner.device)
            self.sums[j : j + 1].add_(v.reshape(1) * weight)

    @torch.no_grad()
    def capture(self, idx: torch.Tensor) -> None:
        learner = self.learner
        cur = torch.cuda.current_stream(learner.device)
        wkey = ("eval", type(learner.model).__name__, self.key[0], self.B, tuple(self.loader.x.shape[1:]))
        with warmup_gate(wkey):  # warm-up (first-use work, creates the sums): alone the first time, then shared
            self.stream.wait_stream(cur)
            with torch.cuda.stream(self.stream):
                self.idx.copy_(idx)
                self.step(self.idx, float(self.B), cache=False)
            self.stream.synchronize()
            gc.collect()  # under the shared gate: never while another thread records
        with GATE.exclusive(), _CAPTURE_LOCK:  # recording only
            torch.cuda.synchronize(learner.device)
            g = torch.cuda.CUDAGraph()
            self.counters = splitk.GraphCounters(learner.device)
            with no_gc(collect=False), splitk.graph_scope(self.counters), torch.cuda.graph(g, stream=self.stream, capture_error_mode="relaxed"):
                self.step(self.idx, float(self.B), cache=False)
            torch.cuda.synchronize(learner.device)
        self.graph = g

    def run(self, idx: torch.Tensor) -> None:
        self.idx.copy_(idx, non_blocking=True)
        assert self.graph is not None
        self.graph.replay()
