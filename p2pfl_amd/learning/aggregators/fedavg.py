"""Federated Averaging (McMahan et al. 2016) on flat arenas.

Reference: ``aggregators/fedavg.py:28-60`` loops ``accum[layer] += m[layer]*w``
over every model and layer (k x L torch ops, re-run for every gossip send).
Here every model is (or is converted to) a :class:`FlatParams` arena and the
whole average is ONE fused HIP kernel (``ops.weighted_average``): k input
pointers, fp32 accumulation, normalisation folded in, 16-byte vector loads,
grid sized for HBM3E bandwidth.  On CPU tensors the same math runs in torch.
"""

from __future__ import annotations

import contextlib
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Tuple

import torch

from p2pfl_amd import ops
from p2pfl_amd.learning.aggregators.aggregator import Aggregator, NoModelsToAggregateError
from p2pfl_amd.learning.arena import FlatParams, flatten, reading
from p2pfl_amd.management.logger import logger
from p2pfl_amd.utils import finite


@dataclass
class _RunningSum:
    """fp32 running sum of the first ``len(keys)`` models in canonical (sorted
    contributor-key) order, raw sample weights, no normalisation yet."""

    acc: torch.Tensor
    layout: Any
    keys: List[str] = field(default_factory=list)
    entries: List[Any] = field(default_factory=list)  # the (model, weight) tuples folded, by identity
    weights: List[float] = field(default_factory=list)


def _reading_all(flats: List[FlatParams]) -> contextlib.ExitStack:
    """``arena.reading`` of every input (the WeightGuard hand-off of live learner weights)."""
    st = contextlib.ExitStack()
    for f in flats:
        st.enter_context(reading(f))
    return st


def _used_here(t: torch.Tensor) -> None:
    """``t`` (allocated on another thread's stream) is read by a kernel about to
    be enqueued on this thread's stream: its block must not be recycled on the
    allocating stream before that kernel ran."""
    if t.is_cuda:
        t.record_stream(torch.cuda.current_stream(t.device))


class FedAvg(Aggregator):
    """Sample-weighted mean of the models.

    Models are folded into a running fp32 sum while the others are still in
    flight (``running_sum``): when a model arrives, every stored model that
    can no longer be preceded in the canonical order by a model still to come
    is added in one fused launch; the aggregation at the end only adds what is
    left and applies ``1 / sum(w)``.  The fold order is the same fixed order
    the one-shot kernel uses, so every node gets the bitwise-same average
    whatever order the models arrived in (``check_equal_models``).
    """

    running_sum = True

    def __init__(self, node_name: str = "unknown") -> None:
        super().__init__(node_name)
        self._run: Optional[_RunningSum] = None

    # -- running sum ----------------------------------------------------------
    # Folds are copy-on-write: a fold writes a NEW accumulator (acc_in = the
    # old one) and installs a new _RunningSum; an accumulator a reader took
    # (aggregate(), a partial aggregation on a gossip thread) is never written
    # again.  Only the planning runs under Aggregator._lock; flattening and the
    # launch run after add_model released it, and the result is published only
    # if the running sum it extends is still the current one.
    def _models_changed_locked(self):
        if not self.running_sum or not self._models:
            self._run = None
            return None
        keys = sorted(self._models)
        run = self._run
        if run is not None and (keys[: len(run.keys)] != run.keys
                                or any(self._models[k] is not e for k, e in zip(run.keys, run.entries))):
            run = self._run = None  # an entry was superseded: the end-of-round aggregation starts over
        have = {n for k in self._models for n in k.split()}
        missing = [n for n in self._train_set if n not in have and n not in self._lost]
        if not missing:
            return None  # complete: aggregate() adds the rest in one launch
        # a future entry is keyed by still-missing names, so it sorts at or
        # after min(missing): everything before that is final in the order
        bound = min(missing)
        start = len(run.keys) if run is not None else 0
        fold = []
        for k in keys[start:]:
            if k >= bound:
                break
            fold.append(k)
        if not fold:
            return None
        entries = [self._models[k] for k in fold]
        return lambda: self._fold(run, fold, entries)

    def _fold(self, base: Optional[_RunningSum], fold: List[str], entries: List[Any]) -> None:
        """Extend ``base`` by ``entries`` into a fresh accumulator (lock NOT held)."""
        ref = entries[0][0]
        device = next(iter(ref.values())).device if len(ref) else torch.device("cpu")
        flats = [flatten(m, device=device) for m, _ in entries]
        layout = base.layout if base is not None else flats[0].layout
        if not all(f.layout.compatible(layout) for f in flats):
            with self._lock:
                if self._run is base:
                    self._run = None
            return
        w = [float(x) for _, x in entries]
        acc = torch.empty(flats[0].flat.numel(), dtype=torch.float32, device=device)
        with logger.span(self.node_name, "fold_models", k=len(fold)), _reading_all(flats):
            if base is not None:
                _used_here(base.acc)
            ops.weighted_sum_into(acc, [f.flat for f in flats], w, acc_in=base.acc if base is not None else None)
        new = _RunningSum(acc, layout,
                          (base.keys if base else []) + fold,
                          (base.entries if base else []) + entries,
                          (base.weights if base else []) + w)
        with self._lock:
            # publish only on top of the sum this fold extended, and only if the
            # folded entries are still the stored ones (a full aggregate or
            # clear() may have replaced them meanwhile)
            if self._run is base and all(self._models.get(k) is e for k, e in zip(new.keys, new.entries)):
                self._run = new

    # -- strategy -------------------------------------------------------------
    def aggregate(self, models: Dict[str, Tuple[Any, int]]) -> FlatParams:
        if len(models) == 0:
            raise NoModelsToAggregateError(f"({self.node_name}) Trying to aggregate models when there is no models")
        # fixed summation order (by contributor key), so every node that
        # aggregates the same models gets the bitwise-same result whatever
        # order they arrived in
        keys = sorted(models)
        entries = [models[k] for k in keys]
        ref = entries[-1][0]
        device = next(iter(ref.values())).device if len(ref) else torch.device("cpu")
        w, scale = ops.fedavg_weights([float(x) for _, x in entries])
        with self._lock:
            run = self._run
            use = (run is not None and keys[: len(run.keys)] == run.keys and run.weights == w[: len(run.keys)]
                   and all(models[k] is e for k, e in zip(run.keys, run.entries)))
            start = len(run.keys) if use else 0
            acc = run.acc if use else None
            layout = run.layout if use else None
        if acc is not None:
            _used_here(acc)  # never written again (copy-on-write folds); keep it alive for this stream
        flats: List[FlatParams] = [flatten(m, device=device) for m, _ in entries[start:]]
        layout = layout if layout is not None else flats[0].layout
        for f in flats:
            if not f.layout.compatible(layout):
                raise ValueError("Cannot average models with different layouts")
        out = torch.empty(flats[0].flat.numel() if flats else acc.numel(), dtype=torch.float32, device=device)
        with _reading_all(flats):  # a learner's live weights: after its last write, before its next
            ops.weighted_sum_into(out, [f.flat for f in flats], w[start:], acc_in=acc, scale=scale)
        if finite.ENABLED:
            for k, f in zip(keys[start:], flats):
                finite.check(self.node_name, "FedAvg input", f, key=k)
            finite.check(self.node_name, "FedAvg running sum", acc, keys=keys[:start])
            finite.check(self.node_name, "FedAvg result", out, keys=keys)
        result = FlatParams.from_flat(out, layout)
        if not isinstance(ref, FlatParams):
            # preserve the caller's key order/names for plain dicts
            renamed = FlatParams()
            for (name, _), view in zip(ref.items(), result.values()):
                renamed[name] = view
            renamed.flat, renamed.layout = result.flat, result.layout
            return renamed
        return result
