"""Partial / full aggregation bookkeeping (reference ``aggregators/aggregator.py:37-281``).

Strategy base: subclasses implement only :meth:`aggregate`.  The base class
tracks which train-set members' models have been folded in and enforces the
decentralised-FedAvg invariant: a stored entry is keyed by its space-joined
contributor list, and a new entry is accepted only if its contributors are all
in the train set and disjoint from every contributor already present (or if it
already covers the whole train set, which replaces everything).

Differences from the reference:

* completion is an ``Event`` instead of a lock released by another thread;
* an empty contributor list returns ``[]`` (Q4: the reference released a lock
  it did not hold and raised);
* a node waiting for the full aggregate that times out with nothing gets
  ``None`` back and keeps its local model (Q5: the reference logged that and
  then raised); missing models are computed from flattened contributors;
* :meth:`would_accept` lets the receive path skip decoding payloads that would
  be rejected anyway;
* partial aggregations are memoised per contributor subset until the stored
  models change (gossip asks for the same subset once per neighbour per
  iteration).
"""

from __future__ import annotations

import threading
from typing import Any, Callable, Dict, List, Optional, Tuple

from p2pfl_amd.management.logger import logger
from p2pfl_amd.settings import Settings
from p2pfl_amd.utils.lockcheck import make_rlock


def _device_work():
    """Shared hold of the process's GPU gate (learning/step_graph.py DeviceGate)
    around aggregation kernels launched from command-handler / gossip threads:
    never beside another virtual peer's HIP-graph capture."""
    from p2pfl_amd.learning.step_graph import GATE

    return GATE.shared()


class NoModelsToAggregateError(Exception):
    """``aggregate`` called with no models."""


ModelEntry = Tuple[Any, int]


class Aggregator:
    def __init__(self, node_name: str = "unknown") -> None:
        self.node_name = node_name
        self._train_set: List[str] = []
        self._waiting_aggregated_model = False
        self._models: Dict[str, ModelEntry] = {}
        self._lock = make_rlock("Aggregator._lock")
        self._done = threading.Event()
        self._running = False
        self._partial_cache: Dict[frozenset, Tuple[Any, List[str], int]] = {}
        # train-set members that left the network mid-round (see mark_lost)
        self._lost: set = set()

    # ------------------------------------------------------------------
    # strategy
    # ------------------------------------------------------------------
    def aggregate(self, models: Dict[str, ModelEntry]) -> Any:
        raise NotImplementedError

    # ------------------------------------------------------------------
    # round control
    # ------------------------------------------------------------------
    def set_nodes_to_aggregate(self, nodes_to_aggregate: List[str]) -> None:
        with self._lock:
            if self._running:
                raise Exception("It is not possible to set nodes to aggregate when the aggregation is running.")
            self._train_set = list(nodes_to_aggregate)
            self._lost = set()
            self._running = True
            self._done.clear()

    def set_waiting_aggregated_model(self, nodes: List[str]) -> None:
        self.set_nodes_to_aggregate(nodes)
        with self._lock:
            self._waiting_aggregated_model = True

    def clear(self) -> None:
        with self._lock:
            self._train_set = []
            self._models = {}
            self._partial_cache = {}
            self._waiting_aggregated_model = False
            self._running = False
            self._lost = set()
            self._models_changed_locked()  # no models: drops any running state, no work to run
            self._done.set()

    def _models_changed_locked(self) -> Optional[Callable[[], None]]:
        """Hook (lock held): the stored models changed and the aggregation is
        not complete yet.  Strategies may start folding them in (FedAvg keeps
        a running sum): the hook only plans under the lock and returns the work
        as a callable, which :meth:`add_model` runs after releasing the lock (so
        flattening / kernel launches never hold up the receive and gossip
        threads).  The default does nothing."""
        return None

    # ------------------------------------------------------------------
    # queries
    # ------------------------------------------------------------------
    def get_aggregated_models(self) -> List[str]:
        with self._lock:
            return [n for key in self._models for n in key.split()]

    @property
    def train_set(self) -> List[str]:
        return list(self._train_set)

    def live_train_set(self) -> List[str]:
        """Train-set members not marked lost: what a full aggregate must cover."""
        with self._lock:
            return [n for n in self._train_set if n not in self._lost]

    def _missing(self) -> List[str]:
        have = set(self.get_aggregated_models())
        return [n for n in self._train_set if n not in have]

    # ------------------------------------------------------------------
    # membership changes (new: the reference waits for a dead train-set
    # member until AGGREGATION_TIMEOUT -- 300 s by default -- and non-members
    # then reject the trainers' aggregate because it lacks that member)
    # ------------------------------------------------------------------
    def mark_lost(self, nodes: List[str]) -> None:
        """Train-set members that left the network: stop waiting for them."""
        with self._lock:
            if not self._running:
                return
            new = (set(nodes) & set(self._train_set)) - self._lost
            if not new:
                return
            self._lost |= new
            logger.info(self.node_name, f"Train-set members lost: {sorted(new)}; aggregating without them")
            if self._complete_locked():
                self._done.set()

    def mark_alive(self, nodes: List[str]) -> None:
        """Train-set members back in the neighbour table (a heartbeat stall, not a
        crash): wait for their models again -- unless the aggregation already
        completed without them, which stays final."""
        with self._lock:
            back = set(nodes) & self._lost
            if not back or self._done.is_set():
                return
            self._lost -= back
            logger.info(self.node_name, f"Train-set members back: {sorted(back)}; waiting for their models again")

    def _complete_locked(self) -> bool:
        if self._waiting_aggregated_model:
            return bool(self._models)
        have = set(self.get_aggregated_models())
        return all(n in have or n in self._lost for n in self._train_set)

    def _full_aggregate_locked(self, contributors: List[str]) -> bool:
        """A diffused model is final if it covers every live train-set member."""
        c = set(contributors)
        return c <= set(self._train_set) and (set(self._train_set) - self._lost) <= c

    def uncovered(self, contributors: List[str]) -> List[str]:
        """Live train-set members a full aggregate with these contributors lacks
        (what keeps a waiting node from accepting it)."""
        with self._lock:
            if not self._waiting_aggregated_model or self._models:
                return []
            c = set(contributors)
            if not c <= set(self._train_set):
                return []
            return [n for n in self._train_set if n not in c and n not in self._lost]

    def would_accept(self, contributors: List[str]) -> bool:
        """Pure version of :meth:`add_model`'s acceptance test."""
        if not contributors:
            return False
        with self._lock:
            if self._waiting_aggregated_model and not self._models:
                return self._full_aggregate_locked(contributors)
            aggregated = self.get_aggregated_models()
            if self._complete_locked():
                return False
            if not all(n in self._train_set for n in contributors):
                return False
            if len(contributors) == len(self._train_set) or self._full_aggregate_locked(contributors):
                return True
            return all(n not in aggregated for n in contributors)

    # ------------------------------------------------------------------
    # model intake
    # ------------------------------------------------------------------
    def add_model(self, model: Any, contributors: List[str], weight: int) -> List[str]:
        nodes = list(contributors)
        if not nodes:
            logger.debug(self.node_name, "Received a model without a list of contributors.")
            return []
        job: List[Optional[Callable[[], None]]] = [None]
        now = self._add_model(model, nodes, weight, job)
        if job[0] is not None:
            with _device_work():
                job[0]()
        return now

    def _add_model(self, model: Any, nodes: List[str], weight: int, job: List[Optional[Callable[[], None]]]) -> List[str]:
        with self._lock:
            if self._waiting_aggregated_model and not self._models:
                if self._full_aggregate_locked(nodes):
                    logger.info(self.node_name, "Received an aggregated model.")
                    self._models = {" ".join(nodes): (model, 1)}
                    self._partial_cache = {}
                    self._waiting_aggregated_model = False
                    self._done.set()
                    return nodes
                return []
            aggregated = self.get_aggregated_models()
            if self._complete_locked():
                logger.debug(self.node_name, "Received a model when is not needed.")
                return []
            if not all(n in self._train_set for n in nodes):
                logger.debug(self.node_name, f"Can't add a model from a node ({nodes}) that is not in the training set.")
                return []
            if len(nodes) == len(self._train_set) or self._full_aggregate_locked(nodes):
                # a full aggregate (of every live member) supersedes the partials
                self._models = {" ".join(nodes): (model, weight)}
            elif all(n not in aggregated for n in nodes):
                self._models[" ".join(nodes)] = (model, weight)
            else:
                logger.debug(self.node_name, f"Can't add a model that has already been added {nodes} / {aggregated}")
                return []
            self._partial_cache = {}
            now = self.get_aggregated_models()
            self._lost -= set(nodes)  # a "lost" member whose model still arrived
            logger.info(self.node_name, f"Model added ({len(now)}/{len(self._train_set)}) from {nodes}")
            if self._complete_locked():
                self._done.set()
            else:
                job[0] = self._models_changed_locked()
            return now

    # ------------------------------------------------------------------
    # results
    # ------------------------------------------------------------------
    def wait_and_get_aggregation(self, timeout: Optional[float] = None) -> Any:
        if timeout is None:
            timeout = Settings.AGGREGATION_TIMEOUT
        self._done.wait(timeout=timeout)
        with self._lock:
            models = dict(self._models)
            waiting = self._waiting_aggregated_model
            train_set = list(self._train_set)
        if waiting:
            if models:
                return next(iter(models.values()))[0]
            logger.info(self.node_name, "Timeout reached by waiting for an aggregated model. Continuing with the local model.")
            return None
        if len(models) == 1 and set(next(iter(models)).split()) == set(train_set):
            return next(iter(models.values()))[0]  # a full aggregate arrived: nothing left to average
        have = {n for key in models for n in key.split()}
        missing = [n for n in train_set if n not in have]
        if missing:
            logger.info(self.node_name, f"Aggregating models, timeout reached. Missing models: {missing}")
        else:
            logger.info(self.node_name, "Aggregating models.")
        if not models:
            return None
        with logger.span(self.node_name, "aggregate", k=len(models)), _device_work():
            return self.aggregate(models)

    def get_partial_aggregation(self, except_nodes: List[str]) -> Tuple[Any, Optional[List[str]], Optional[int]]:
        excl = set(except_nodes)
        with self._lock:
            chosen = {k: v for k, v in self._models.items() if not (set(k.split()) & excl)}
            if not chosen:
                return None, None, None
            key = frozenset(chosen)
            hit = self._partial_cache.get(key)
            if hit is not None:
                return hit
        contributors = [n for k in chosen for n in k.split()]
        weight = sum(w for _, w in chosen.values())
        if len(chosen) == 1:
            result = (next(iter(chosen.values()))[0], contributors, weight)
        else:
            with logger.span(self.node_name, "partial_aggregate", k=len(chosen)), _device_work():
                result = (self.aggregate(chosen), contributors, weight)
        with self._lock:
            if all(k in self._models for k in chosen):
                self._partial_cache[key] = result
        return result
