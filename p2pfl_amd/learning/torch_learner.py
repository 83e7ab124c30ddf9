"""PyTorch-ROCm learner (reference ``learning/pytorch/lightning_learner.py:45-236``).

Replaces the Lightning ``Trainer`` with an explicit loop tuned for MI355X:

* the model's parameters, buffers and gradients are re-homed into flat arenas
  (:class:`~p2pfl_amd.learning.arena.ModuleArena`), so ``get_parameters`` is
  zero-copy, ``set_parameters`` is one device copy, gossip snapshots are one
  ``clone`` and FedAvg is one kernel;
* when the model's ``configure_optimizers`` returns plain Adam/SGD over all
  parameters, the step runs as ONE fused HIP kernel over the whole arena
  (``ops.adam_step`` / ``ops.sgd_step``) instead of per-tensor launches;
* data batches are produced on the device (no loader workers);
* compute runs under bf16 autocast on the GPU (fp32 master weights and
  optimizer state), fp32 on the CPU.  On the GPU the matrix weights are bf16
  views of a shadow arena rewritten by the optimizer kernel (``mixed``), and
  gradients stay per-tensor (bf16 for bf16 weights) and are consumed by ONE
  multi-tensor Adam/SGD launch -- no per-weight cast, zero-fill or
  accumulate kernels in the step;
* the optimizer is re-created on every :meth:`fit`, as Lightning does when a
  new ``Trainer`` is built per round (reference quirk Q23, kept).

Metrics: per-step ``train_loss`` (every ``log_every_n_steps``) and per-epoch
validation metrics go to the local store, ``evaluate`` results to the global
store, exactly where the reference's ``FederatedLogger`` put them.
"""

from __future__ import annotations

import os
import contextlib
import threading
import time
from collections import OrderedDict
from typing import Any, Dict, Mapping, Optional, Tuple

import torch

from p2pfl_amd.data.datamodule import wants_float

from p2pfl_amd import ops
from p2pfl_amd.learning.arena import FlatParams, ModuleArena
from p2pfl_amd.learning.exceptions import DecodingParamsError, ModelNotMatchingError
from p2pfl_amd.learning.learner import NodeLearner
from p2pfl_amd.learning.wire import decode_params, encode_params
from p2pfl_amd.management.logger import logger
from p2pfl_amd.utils.streams import private_stream
from p2pfl_amd.settings import Settings
from p2pfl_amd.utils import finite

# queue priority of the learners' compute streams (P2PFL_COMPUTE_STREAM_PRIORITY: -1 highest,
# 0 default; measurement knob -- the evaluation streams sit at the lowest priority)
_COMPUTE_PRIORITY = int(os.environ.get("P2PFL_COMPUTE_STREAM_PRIORITY", "0"))
# A/B switches (read once): graphs for an epoch's short last batch, and
# evaluation passes whose metrics are read back by a completion thread
_TAIL_GRAPHS = os.environ.get("P2PFL_TAIL_GRAPHS", "1") != "0"
_ASYNC_EVAL = os.environ.get("P2PFL_ASYNC_EVAL", "1") != "0"


def default_device() -> torch.device:
    return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")


class TorchLearner(NodeLearner):
    def __init__(
        self,
        model: Any,
        data: Any,
        self_addr: str,
        epochs: int,
        device: Optional[torch.device] = None,
        precision: Optional[str] = None,
        log_every_n_steps: int = 50,
        fused_optimizer: bool = True,
        mixed: Optional[bool] = None,
        use_step_graphs: bool = True,
    ) -> None:
        if Settings.TORCH_NUM_THREADS:
            torch.set_num_threads(Settings.TORCH_NUM_THREADS)
        self._addr = self_addr
        self.epochs = epochs
        self.device = torch.device(device) if device is not None else default_device()
        if self.device.type == "cuda":
            # MIOpen "find" mode: benchmark the solvers once per conv shape.
            # Without it several ResNet shapes fall back to MIOpen's naive
            # kernels (77 % of a ResNet-18 round on MI355X).
            torch.backends.cudnn.benchmark = True
            # pre-tuned hipBLASLt/rocBLAS GEMM selections (p2pfl_amd/tuning)
            from p2pfl_amd.tuning import enable_tuned_gemms

            enable_tuned_gemms()
        self.precision = precision or ("bf16" if self.device.type == "cuda" else "fp32")
        self.log_every_n_steps = log_every_n_steps
        self.fused_optimizer = fused_optimizer
        self._mixed_opt = mixed
        self.mixed = False
        self._interrupt = threading.Event()
        self._step = 0
        from p2pfl_amd.learning.federated_logger import FederatedLogger

        # per-step metric sink (reference: the Lightning logger plugged into the Trainer)
        self.metrics_logger = FederatedLogger(self_addr)
        # HIP-graph replay of the training step (mixed precision, device-resident data)
        self.use_step_graphs = use_step_graphs and os.environ.get("P2PFL_STEP_GRAPHS", "1") != "0"
        self._mt_opt: Any = None
        self._arena_version = 0
        self._snapshot: Optional[Tuple[int, FlatParams]] = None
        # this node's compute stream (Settings.NODE_STREAMS): virtual peers in
        # one process train concurrently, and their training overlaps the
        # aggregation / transport work left on the default stream
        self._compute_stream: Optional[torch.cuda.Stream] = None
        self._step_graph: Any = None
        self._tail_graphs: Dict[int, Any] = {}  # short last batch of an epoch, by size
        self._eval_graphs: Dict[str, Any] = {}
        self._completions: Any = None  # metric read-backs of asynchronous evaluation passes
        self.model: Any = None
        self.arena: Optional[ModuleArena] = None
        self.data: Any = None
        self.set_model(model)
        self.set_data(data)

    # ------------------------------------------------------------------
    # model / data
    # ------------------------------------------------------------------
    def set_model(self, model: Any) -> None:
        self.model = model
        if model is None:
            self.arena = None
            return
        model.to(self.device)
        self.mixed = self._want_mixed(model)
        if self.mixed:
            keep = model.fp32_parameter_names() if hasattr(model, "fp32_parameter_names") else None
            cl = model.channels_last_parameter_names() if hasattr(model, "channels_last_parameter_names") else None
            self.arena = ModuleArena(model, device=self.device, compute_dtype=torch.bfloat16, fp32_names=keep, channels_last_names=cl)
        else:
            self.arena = ModuleArena(model, device=self.device, grads=True)

    def _want_mixed(self, model: Any) -> bool:
        """bf16 weight shadows + multi-tensor optimizer (GPU, bf16, fusable optimizer)."""
        if self._mixed_opt is not None:
            return bool(self._mixed_opt)
        if not (self.device.type == "cuda" and self.precision == "bf16" and self.fused_optimizer and ops.available()):
            return False
        from p2pfl_amd.learning.optim import fusable

        opt = model.configure_optimizers()
        return fusable(opt[0] if isinstance(opt, (list, tuple)) else opt, model)

    def set_data(self, data: Any) -> None:
        self.data = data
        if data is not None and hasattr(data, "to"):
            data.to(self.device)

    def get_num_samples(self) -> Tuple[int, int]:
        return (len(self.data.train_dataloader().dataset), len(self.data.test_dataloader().dataset))

    # ------------------------------------------------------------------
    # parameters
    # ------------------------------------------------------------------
    def get_parameters(self) -> FlatParams:
        """The live weights (no copy), safe to read on the caller's current stream:
        it waits for the learner's last write, and the learner's next write waits
        for what the caller queued on it meanwhile (WeightGuard ``hand_out``)."""
        params = self.live_parameters()
        guard = self._guard()
        if guard is not None and self.device.type == "cuda":
            guard.hand_out(torch.cuda.current_stream(self.device))
        return params

    def live_parameters(self) -> FlatParams:
        """The live weights with no stream ordering: the framework's own consumers
        (FedAvg, gossip snapshots, encoding) launch their reads under
        ``arena.reading(params)``, which orders exactly those reads (the
        :class:`~p2pfl_amd.learning.arena.WeightGuard` the arena carries) -- a
        lone trainer's round then pays no cross-queue wait."""
        assert self.arena is not None
        if self.arena._int_buffers:
            # integer-buffer mirror copies (BatchNorm counters): a write of the
            # arena on the caller's stream, after the learner's last block
            guard = self._guard()
            cur = torch.cuda.current_stream(self.device) if self.device.type == "cuda" else None
            with self._gate():
                if guard is not None:
                    guard.begin_write(cur)
                self.arena.sync_in()
                if guard is not None:
                    guard.end_write(cur)
        return self.arena.params

    def _guard(self):
        return getattr(self.arena.params, "guard", None) if self.arena is not None else None

    def _stream_for_block(self) -> Optional[torch.cuda.Stream]:
        """This learner's compute stream (``Settings.NODE_STREAMS``; ``"auto"``: every
        GPU learner), or None to enqueue on the caller's stream.  The hand-offs to
        the threads that read the weights on other streams are lazy (the arena's
        WeightGuard): a block waits only for reads / writes launched elsewhere
        since the last one, so a lone trainer pays no cross-queue wait at all."""
        if self.device.type != "cuda" or not Settings.NODE_STREAMS:
            return None
        if self._compute_stream is None:
            self._compute_stream = private_stream(self.device, _COMPUTE_PRIORITY)
        return self._compute_stream

    @contextlib.contextmanager
    def _on_stream(self, hold_gate: bool = False, wait_caller: bool = False, writes: bool = True):
        """Run a block on this learner's compute stream.

        Ordering, without host synchronisation and without handing the stream back
        to the caller's (``profiles/r5_handoff_probe.md``: every such hand-back cost
        the next epoch ~0.55 ms of device time):

        * ``writes`` (fit, set_parameters): the block starts after every read of the
          weights launched on other streams since the last write (FedAvg folds,
          gossip snapshots -- WAR), and records the weights' ready event at its end,
          which readers on other streams wait on where they launch (RAW);
        * otherwise (evaluation) the block only waits for the last write if that ran
          on another stream;
        * ``wait_caller``: the block also consumes something the caller's stream
          produced (``set_parameters`` copying an aggregate the FedAvg kernel wrote
          there): the compute stream first waits for the caller's stream.

        ``hold_gate``: the whole block is short GPU work issued from a non-learning
        thread (set_parameters from a command handler): it runs under the shared
        device gate, never beside another peer's capture (a copy launched from a
        handler thread during a capture crashed the HIP runtime once under rocprofv3
        in the 8-peer scenario).
        """
        cs = self._stream_for_block()
        cur = torch.cuda.current_stream(self.device) if self.device.type == "cuda" else None
        run = cs if cs is not None else cur
        guard = self._guard()
        gate = self._gate() if hold_gate else contextlib.nullcontext()
        from p2pfl_amd.learning.step_graph import GATE

        if wait_caller and cs is not None and cur != cs:
            # recorded on the caller's stream -- usually the legacy default stream,
            # which ROCm treats as part of a capture in progress on another peer's
            # thread (hipErrorCapturedEvent): never while another thread captures
            with GATE.shared():
                cs.wait_stream(cur)
        if guard is not None:
            if writes:
                guard.begin_write(run)
            else:
                guard.acquire(run)
        try:
            with gate, (torch.cuda.stream(cs) if (cs is not None and cur != cs) else contextlib.nullcontext()):
                yield
        finally:
            if writes and guard is not None:
                guard.end_write(run)

    def set_parameters(self, params: Mapping[str, torch.Tensor]) -> None:
        finite.check(self._addr, "set_parameters input", params if isinstance(params, FlatParams) else None)
        if (self.arena is not None and isinstance(params, FlatParams)
                and params.flat.data_ptr() == self.arena.params.flat.data_ptr()):
            self._arena_changed()
            return  # the arena itself (a one-member aggregate): no copy, so no stream hand-off either
        with self._on_stream(hold_gate=True, wait_caller=True):
            self._set_parameters(params)
            cs = self._stream_for_block()
            if cs is not None:
                # the source (an aggregate or a received model, allocated on another
                # stream) is read by this stream's copy: no hand-back orders its
                # release after the copy, so tell the caching allocator
                srcs = [params.flat] if isinstance(params, FlatParams) else list(params.values())
                for t in srcs:
                    if isinstance(t, torch.Tensor) and t.is_cuda:
                        t.record_stream(cs)
        if finite.ENABLED and self.arena is not None:
            finite.check(self._addr, "parameters after set_parameters", self.arena.flat)

    def _set_parameters(self, params: Mapping[str, torch.Tensor]) -> None:
        assert self.arena is not None
        self._arena_changed()
        own = self.arena.params
        if isinstance(params, FlatParams) and params.flat.data_ptr() == own.flat.data_ptr():
            return  # the arena itself (e.g. a one-member aggregate): nothing to copy
        try:
            if isinstance(params, FlatParams) and params.layout.compatible(own.layout):
                own.flat.copy_(params.flat, non_blocking=True)
            else:
                if len(params) != len(own):
                    raise ModelNotMatchingError(f"expected {len(own)} tensors, got {len(params)}")
                # names may differ (positional compatibility), shapes must not
                for (name, dst), src in zip(own.items(), params.values()):
                    if tuple(src.shape) != tuple(dst.shape):
                        raise ModelNotMatchingError(f"shape mismatch for {name}: {tuple(src.shape)} vs {tuple(dst.shape)}")
                    dst.copy_(src.reshape(dst.shape), non_blocking=True)
            self.arena.sync_out()
        except ModelNotMatchingError:
            raise
        except Exception as e:
            raise ModelNotMatchingError("Not matching models") from e

    def encode_parameters(self, params: Optional[Mapping[str, torch.Tensor]] = None) -> bytes:
        if params is None:
            params = self.live_parameters()
        from p2pfl_amd.learning.arena import reading

        with reading(params):
            return encode_params(params)

    def snapshot_parameters(self, params: Optional[Mapping[str, torch.Tensor]] = None) -> FlatParams:
        """Immutable device payload for gossip.

        Only the LIVE arena changes under a payload (training, set_parameters),
        so only it is copied -- once per arena version, shared by every
        neighbour and gossip iteration until the arena changes.  Aggregates and
        received models are fresh buffers nobody mutates: they go out as is.
        """
        if params is None:
            params = self.live_parameters()
        if isinstance(params, FlatParams):
            if self.arena is None or params.flat.data_ptr() != self.arena.flat.data_ptr():
                return params
            snap = self._snapshot
            if snap is None or snap[0] != self._arena_version:
                from p2pfl_amd.learning.arena import reading

                # a copy launched from a gossip thread: never beside a capture; after
                # the last write of the weights, before the next (WeightGuard)
                with self._gate(), reading(params):
                    snap = self._snapshot = (self._arena_version, params.clone())
            return snap[1]
        from p2pfl_amd.learning.arena import flatten

        return flatten(params, device=self.device)

    def _arena_changed(self) -> None:
        self._arena_version += 1
        self._snapshot = None

    def decode_parameters(self, data: Any) -> FlatParams:
        assert self.arena is not None
        try:
            if isinstance(data, FlatParams):
                params = data.to(self.device, non_blocking=True)
            elif isinstance(data, (bytes, bytearray, memoryview)):
                params = decode_params(data)
                if isinstance(params, FlatParams):
                    params = params.to(self.device)
            else:
                raise DecodingParamsError(f"unsupported payload type {type(data).__name__}")
        except DecodingParamsError:
            raise
        except Exception as e:
            raise DecodingParamsError("Error decoding parameters") from e
        own = self.arena.params
        if isinstance(params, FlatParams):
            if not params.layout.compatible(own.layout):
                raise ModelNotMatchingError("payload layout does not match the local model")
            return FlatParams.from_flat(params.flat, own.layout)
        if isinstance(params, list):
            # the reference's positional [ndarray, ...] (state_dict order); its
            # zip() silently truncated on a count mismatch (quirk Q17): checked here
            if len(params) != len(own) or any(
                tuple(a.shape) != tuple(b.shape) for a, b in zip(params, own.values())
            ):
                raise ModelNotMatchingError("reference payload does not match the local model")
            params = OrderedDict(zip(own.keys(), params))
        # generic dict payload: validate then re-home
        if len(params) != len(own) or any(tuple(a.shape) != tuple(b.shape) for a, b in zip(params.values(), own.values())):
            raise ModelNotMatchingError("payload tensors do not match the local model")
        flat = torch.zeros_like(own.flat)
        out = FlatParams.from_flat(flat, own.layout)
        for dst, src in zip(out.values(), params.values()):
            dst.copy_(src.reshape(dst.shape))
        return out

    # ------------------------------------------------------------------
    # training
    # ------------------------------------------------------------------
    def set_epochs(self, epochs: int) -> None:
        self.epochs = epochs

    def _autocast(self):
        if self.precision == "bf16":
            return torch.autocast(device_type=self.device.type, dtype=torch.bfloat16)
        return torch.autocast(device_type="cpu", enabled=False)

    def _make_optimizer(self):
        opt = self.model.configure_optimizers()
        if isinstance(opt, (list, tuple)):
            opt = opt[0]
        if self.mixed:
            from p2pfl_amd.learning.optim import fuse_optimizer_mt

            fused = fuse_optimizer_mt(opt, self.arena)
            if fused is None:  # bf16 weights must not be stepped by torch.optim
                raise RuntimeError("mixed-precision learner needs a plain Adam/AdamW/SGD over all parameters")
            prev = self._mt_opt
            if prev is not None and prev.arena is self.arena and prev.config() == fused.config():
                # same optimizer re-created: reset the persistent one instead
                # (identical state, and a captured step graph stays valid)
                prev.reset()
                return prev
            self._mt_opt = fused
            return fused
        if not (self.fused_optimizer and self.device.type == "cuda" and self.arena is not None):
            return opt
        from p2pfl_amd.learning.optim import fuse_optimizer

        return fuse_optimizer(opt, self.arena) or opt

    def interrupt_fit(self) -> None:
        self._interrupt.set()

    def fit(self) -> None:
        if self.epochs <= 0 or self.model is None:
            return
        if finite.ENABLED and self.arena is not None:
            finite.check(self._addr, "parameters before fit", self.arena.flat)
        try:
            with self._on_stream():
                self._fit()
        finally:
            # a snapshot taken while fit() ran (weights still moving) must not
            # be served as the trained model's payload
            self._arena_changed()
        if finite.ENABLED and self.arena is not None:
            finite.check(self._addr, "parameters after fit", self.arena.flat, step=self._step)

    def _fit(self) -> None:
        self._interrupt.clear()
        self._arena_changed()
        try:
            opt = self._make_optimizer()
            model = self.model
            for _epoch in range(self.epochs):
                model.train()
                loader = self.data.train_dataloader()
                if self._graph_ok(opt, loader):
                    cur = torch.cuda.current_stream(self.device)
                    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    t0.record(cur)
                    with logger.span(self._addr, "train_epoch"):
                        if not self._fit_epoch_graph(opt, loader):
                            return
                    t1.record(cur)
                    self._validate()
                    self._record_epoch_gpu(t0, t1)
                    continue
                with logger.span(self._addr, "train_epoch"):
                    for i, batch in enumerate(loader):
                        if self._interrupt.is_set():
                            return
                        with self._gate():
                            opt.zero_grad(set_to_none=False)
                            with self._autocast():
                                loss = model.training_step(batch, i)
                            loss.backward()
                            opt.step()
                            del loss
                        self._step += 1
                        if self.log_every_n_steps and self._step % self.log_every_n_steps == 0:
                            for k, v in model.pop_logged().items():
                                self._log(k, float(v), step=self._step)
                if self.arena is not None and not self.arena.grads_bound():
                    self.arena.rebind_grads()
                self._validate()
        except Exception as e:
            logger.error(self._addr, f"Fit error: {e}")
            raise

    def _record_epoch_gpu(self, t0: Any, t1: Any) -> None:
        """Device time of the epoch just enqueued ("train_epoch_gpu") and from the
        previous epoch's end to its start ("inter_epoch_gpu": evaluation passes,
        host hand-offs, idle time) -- read without a host sync of its own: the
        events are resolved when the NEXT epoch records them (bench.py spans)."""
        prev = getattr(self, "_epoch_events", None)
        self._epoch_events = (t0, t1)
        if prev is None or not prev[1].query():
            return
        now = time.perf_counter()
        ms = prev[0].elapsed_time(prev[1])
        logger.tracer.record(self._addr, "train_epoch_gpu", now - ms * 1e-3, ms * 1e-3)
        gap = prev[1].elapsed_time(t0)
        logger.tracer.record(self._addr, "inter_epoch_gpu", now - gap * 1e-3, gap * 1e-3)

    def _gate(self):
        """Shared hold of the process's GPU gate around one step / eval pass (see step_graph.DeviceGate)."""
        if self.device.type != "cuda":
            return contextlib.nullcontext()
        from p2pfl_amd.learning.step_graph import GATE

        return GATE.shared()

    def _graph_ok(self, opt: Any, loader: Any) -> bool:
        if not (self.use_step_graphs and self.mixed and self.device.type == "cuda" and hasattr(opt, "step_graph")):
            return False
        from p2pfl_amd.learning.step_graph import graphable_loader

        return graphable_loader(loader)

    def _fit_epoch_graph(self, opt: Any, loader: Any) -> bool:
        """One epoch with full batches replayed from a captured step graph; False if interrupted."""
        from p2pfl_amd.learning.step_graph import TrainStepGraph

        model = self.model
        B, n = int(loader.batch_size), len(loader.dataset)
        # the same batch order as iterating the loader.  A pinned host buffer and an H2D
        # copy: under the shared gate, never beside another peer's capture (the host
        # allocator queries events that may have been recorded in a capturing stream:
        # hipErrorCapturedEvent, scripts/repro_virtual_peers.py)
        with self._gate():
            perm = loader.permutation()
        key = TrainStepGraph.make_key(self, opt, loader)
        for i, s in enumerate(range(0, n, B)):
            if self._interrupt.is_set():
                return False
            idx = perm[s : s + B]
            # every full batch replays the graph, the fit's first one too when the optimizer's
            # graph step on its reset state equals the eager first step (Adam; SGD without
            # dampening): no eager step -- ~200 host-side launches -- per fit
            first_ok = opt.t >= 1 or (hasattr(opt, "graph_first_step_ok") and opt.graph_first_step_ok())
            if idx.numel() == B and first_ok:
                sg = self._step_graph
                if sg is None or sg.key != key:
                    sg = self._step_graph = TrainStepGraph(self, opt, loader)
                    sg.capture(idx)  # takes the gate exclusively
                with self._gate():
                    logged = {"train_loss": sg.run(idx)}
            elif first_ok and idx.numel() > 1 and _TAIL_GRAPHS:
                # the epoch's short last batch: a graph of its own size (captured once; the
                # same remainder every epoch) instead of ~200 eager launches per round
                nb = int(idx.numel())
                tg = self._tail_graphs.get(nb)
                if tg is None or tg.key != TrainStepGraph.make_key(self, opt, loader, nb):
                    tg = self._tail_graphs[nb] = TrainStepGraph(self, opt, loader, nb)
                    tg.capture(idx)
                with self._gate():
                    logged = {"train_loss": tg.run(idx)}
            else:  # first step when it must seed optimizer state eagerly (and a one-sample batch)
                with self._gate():
                    x = loader.x.index_select(0, idx)
                    if wants_float(loader, model):
                        x = x.float().div_(255.0)
                    opt.zero_grad(set_to_none=True)
                    with self._autocast():
                        loss = model.training_step((x, loader.y.index_select(0, idx)), i)
                    loss.backward()
                    opt.step()
                    # drop this step's autograd graph now: its AccumulateGrad nodes
                    # (bound to this stream) must not survive into a graph capture
                    del loss
                    logged = model.pop_logged()
            self._step += 1
            if self.log_every_n_steps and self._step % self.log_every_n_steps == 0:
                for k, v in logged.items():
                    self._log(k, float(v), step=self._step)
        return True

    @torch.no_grad()
    def _run_eval(self, loader, hook) -> Dict[str, float]:
        self.model.eval()
        if self._eval_graph_ok(loader):
            return self._run_eval_graph(loader, hook)
        with self._gate():
            return self._run_eval_eager(loader, hook)

    def _run_eval_eager(self, loader, hook) -> Dict[str, float]:
        sums: Dict[str, torch.Tensor] = {}
        n = 0
        for i, (x, y) in enumerate(loader):
            with self._autocast():
                hook((x, y), i)
            bs = int(y.shape[0])
            for k, v in self.model.pop_logged().items():
                v = v.float() if isinstance(v, torch.Tensor) else torch.tensor(float(v))
                sums[k] = sums.get(k, 0) + v * bs
            n += bs
        return {k: float(v) / max(1, n) for k, v in sums.items()}

    def validate(self) -> None:
        """The per-epoch validation pass (metrics to the local store)."""
        with self._on_stream(writes=False):
            self._validate()

    def _eval_graph_ok(self, loader: Any) -> bool:
        if not (self.use_step_graphs and self.mixed and self.device.type == "cuda"):
            return False
        from p2pfl_amd.learning.step_graph import graphable_loader

        return graphable_loader(loader) and len(loader.dataset) >= loader.batch_size

    @staticmethod
    def _eval_batch(loader: Any) -> int:
        """Samples per captured evaluation step: ``Settings.EVAL_BATCH_FACTOR`` x the
        loader's batch, halved until it fits the set.  Evaluation has no optimizer
        step and BatchNorm uses its running statistics, so per-sample losses and
        predictions -- and the pass's means -- do not depend on the batching; the
        larger products (ViT-B: M = 4 x 6304 tokens) run at a higher MFMA rate."""
        from p2pfl_amd.settings import Settings

        bs, n = int(loader.batch_size), len(loader.dataset)
        k = max(1, int(Settings.EVAL_BATCH_FACTOR))
        while k > 1 and bs * k > n:
            k //= 2
        return bs * k

    def _run_eval_graph(self, loader: Any, hook: Any, on_done: Any = None) -> Optional[Dict[str, float]]:
        """Full batches replay a captured evaluation graph; sums stay on the device.
        With ``on_done`` the pass is only enqueued: the sums are read back into
        pinned memory behind it and ``on_done(metrics)`` runs on the completion
        thread when they land (no host sync; returns None)."""
        from p2pfl_amd.learning.step_graph import EvalStepGraph

        B, n = self._eval_batch(loader), len(loader.dataset)
        name = getattr(hook, "__name__", str(hook))
        key = EvalStepGraph.make_key(self, loader, hook, B)
        eg = self._eval_graphs.get(name)
        with self._gate():  # pinned host buffer + H2D copy: never beside another peer's capture
            perm = loader.permutation()
        if eg is None or eg.key != key:
            eg = self._eval_graphs[name] = EvalStepGraph(self, loader, hook, B)
            eg.capture(perm[:B])  # takes the gate exclusively
        tail = n % B
        tg = None
        if tail > 1:  # the set's remainder: a graph of its own size, accumulating into the same sums
            tkey = ("tail",) + EvalStepGraph.make_key(self, loader, hook, tail)
            tg = self._eval_graphs.get(name + "/tail")
            if tg is None or tg.key != tkey:
                tg = self._eval_graphs[name + "/tail"] = EvalStepGraph(self, loader, hook, tail, sums_of=eg)
                tg.key = tkey
                tg.capture(perm[n - tail:])
        with self._gate():
            eg.sums.zero_()
            for s in range(0, n, B):
                idx = perm[s : s + B]
                if idx.numel() == B:
                    eg.run(idx)
                elif tg is not None:
                    tg.run(idx)
                else:
                    eg.step(idx, float(idx.numel()))
            if on_done is not None:
                host = torch.empty(eg.sums.shape, dtype=eg.sums.dtype, pin_memory=True)
                host.copy_(eg.sums, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(torch.cuda.current_stream(self.device))
            else:
                vals = eg.sums.tolist()
        if on_done is not None:
            keys = list(eg.keys)
            if self._completions is None:
                from p2pfl_amd.learning.host_completion import HostCompletions

                self._completions = HostCompletions(self._addr)
            self._completions.submit(ev, lambda: on_done({k: v / max(1, n) for k, v in zip(keys, host.tolist())}))
            return None
        return {k: v / max(1, n) for k, v in zip(eg.keys, vals)}

    def _validate(self) -> None:
        loader = self.data.val_dataloader()
        if loader is None or len(loader.dataset) == 0:
            return
        step = self._step
        if _ASYNC_EVAL and self._eval_graph_ok(loader):  # metrics logged when they land; the next epoch is already queued
            self.model.eval()
            self._run_eval_graph(loader, self.model.validation_step,
                                 lambda res: [self._log(k, v, step=step) for k, v in res.items()])
            return
        for k, v in self._run_eval(loader, self.model.validation_step).items():
            self._log(k, v, step=step)

    def evaluate_async(self, on_results: Any = None) -> bool:
        """Graph-replayed test pass enqueued on the node's stream (ahead of the next
        fit, which the stream orders after it); metrics are logged and handed to
        ``on_results`` by the completion thread.  False (use :meth:`evaluate`)
        where the pass would run eagerly."""
        if self.epochs <= 0 or self.model is None:
            return False
        loader = self.data.test_dataloader()
        if not (_ASYNC_EVAL and self._eval_graph_ok(loader)):
            return False

        def done(results: Dict[str, float]) -> None:
            for k, v in results.items():
                self._log(k, v)
            if on_results is not None:
                on_results(results)

        with logger.span(self._addr, "evaluate"), self._on_stream(writes=False):
            self.model.eval()
            self._run_eval_graph(loader, self.model.test_step, done)
        return True

    def drain(self, timeout: Optional[float] = None) -> bool:
        return self._completions.drain(timeout) if self._completions is not None else True

    def evaluate(self) -> Dict[str, float]:
        if self.epochs <= 0 or self.model is None:
            return {}
        box: Dict[str, float] = {}
        if self.evaluate_async(box.update):
            self.drain()
            return box
        with logger.span(self._addr, "evaluate"), self._on_stream(writes=False):
            results = self._run_eval(self.data.test_dataloader(), self.model.test_step)
        for k, v in results.items():
            self._log(k, v)
        return results

    def _log(self, key: str, value: float, step=None) -> None:
        """Per-step metrics go through the FederatedLogger adapter (as the
        reference's Trainer logger did, ``lightning_logger.py:54-57``); round
        metrics (no step) straight to the global store."""
        try:
            if step is not None:
                self.metrics_logger.log_metrics({key: value}, step)
            else:
                logger.log_metric(self._addr, key, value)
        except Exception:
            pass  # learner used outside a registered node (benchmarks, unit tests)


# Reference-compatible name: users of ``LightningLearner`` keep their imports.
LightningLearner = TorchLearner
