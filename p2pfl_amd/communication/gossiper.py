"""Gossip engine (reference ``communication/gossiper.py:31-243``).

Two independent jobs:

1. **Control-message relay** (thread).  Flooded messages with ``ttl > 1`` are
   queued with the list of neighbours still to receive them and sent at most
   ``GOSSIP_MESSAGES_PER_PERIOD`` per ``GOSSIP_PERIOD``.  The thread sleeps on
   a condition variable while the queue is empty (the reference busy-polls,
   with ``GOSSIP_PERIOD = 0`` in tests).
2. **Model gossip** (:meth:`gossip_weights`, runs in the caller's thread).
   Push partial/full aggregates to candidates chosen by callbacks until no
   candidate is left, the caller stops, or the status stalls.

Event-driven model gossip: the loop waits on the node's
:class:`~p2pfl_amd.node_state.ChangeSignal`, so an iteration starts as soon as
a peer acknowledges (``models_aggregated`` / ``models_ready``) instead of after
a fixed ``GOSSIP_MODELS_PERIOD`` sleep.  A neighbour is re-sent a model only if
the node state changed since the previous send to it or a full period passed,
so wake-ups never turn into duplicate multi-MB pushes.

Reference quirks fixed: the periodic sleep is ``period - elapsed`` (Q1), and
the stall exit requires ``GOSSIP_EXIT_ON_X_EQUAL_ROUNDS`` identical snapshots
taken at least one period apart (Q2).
"""

from __future__ import annotations

import collections
import random
import threading
import time
from typing import Any, Callable, Deque, Dict, List, Optional, Set, Tuple

from p2pfl_amd.management.logger import logger
from p2pfl_amd.settings import Settings
from p2pfl_amd.utils.lockcheck import make_condition, make_lock


class Gossiper(threading.Thread):
    def __init__(
        self,
        self_addr: str,
        client: Any,
        period: Optional[float] = None,
        messages_per_period: Optional[int] = None,
    ) -> None:
        super().__init__(name=f"gossiper-thread-{self_addr}", daemon=True)
        self._self_addr = self_addr
        self._client = client
        self.period = Settings.GOSSIP_PERIOD if period is None else period
        self.messages_per_period = (
            Settings.GOSSIP_MESSAGES_PER_PERIOD if messages_per_period is None else messages_per_period
        )
        # duplicate suppression: O(1) membership + FIFO eviction
        self._seen: Set[int] = set()
        self._seen_order: Deque[int] = collections.deque()
        self._seen_lock = make_lock("Gossiper._seen_lock")
        # relay queue
        self._pending: Deque[Tuple[Any, List[str]]] = collections.deque()
        self._cv = make_condition("Gossiper._cv")
        self._terminate = threading.Event()

    # ------------------------------------------------------------------
    # thread control
    # ------------------------------------------------------------------
    def stop(self) -> None:
        self._terminate.set()
        with self._cv:
            self._cv.notify_all()

    # ------------------------------------------------------------------
    # relay
    # ------------------------------------------------------------------
    def add_message(self, msg: Any, pending_neis: List[str]) -> None:
        if not pending_neis:
            return
        with self._cv:
            self._pending.append((msg, list(pending_neis)))
            self._cv.notify()

    def check_and_set_processed(self, msg_hash: int) -> bool:
        """True the first time a hash is seen (then remembered), False after."""
        with self._seen_lock:
            if msg_hash in self._seen:
                return False
            self._seen.add(msg_hash)
            self._seen_order.append(msg_hash)
            while len(self._seen_order) > Settings.AMOUNT_LAST_MESSAGES_SAVED:
                self._seen.discard(self._seen_order.popleft())
            return True

    def _take_batch(self) -> List[Tuple[Any, List[str]]]:
        batch: List[Tuple[Any, List[str]]] = []
        budget = self.messages_per_period
        while budget > 0 and self._pending:
            msg, neis = self._pending[0]
            if len(neis) <= budget:
                batch.append((msg, neis))
                self._pending.popleft()
                budget -= len(neis)
            else:
                batch.append((msg, neis[:budget]))
                self._pending[0] = (msg, neis[budget:])
                budget = 0
        return batch

    def run(self) -> None:
        while not self._terminate.is_set():
            t0 = time.monotonic()
            with self._cv:
                while not self._pending and not self._terminate.is_set():
                    self._cv.wait(timeout=0.5)
                batch = self._take_batch()
            for msg, neis in batch:
                for nei in neis:
                    if self._terminate.is_set():
                        return
                    self._client.send(nei, msg)
            # rate limit only when the budget was exhausted
            if self.period > 0 and sum(len(n) for _, n in batch) >= self.messages_per_period:
                self._terminate.wait(max(0.0, self.period - (time.monotonic() - t0)))

    # ------------------------------------------------------------------
    # model gossip (synchronous)
    # ------------------------------------------------------------------
    def gossip_weights(
        self,
        early_stopping_fn: Callable[[], bool],
        get_candidates_fn: Callable[[], List[str]],
        status_fn: Callable[[], Any],
        model_fn: Callable[[str], Any],
        period: float,
        create_connection: bool,
        wakeup: Any = None,
        peer_status_fn: Optional[Callable[[str], Any]] = None,
    ) -> None:
        """Push models until no candidate is left.

        A candidate is (re)sent a model when it has never been sent one, when
        ITS status (``peer_status_fn(n)``: what it reported having) changed
        since the last send to it, or when a full ``period`` passed -- other
        peers' reports waking the loop never cause duplicate multi-MB pushes
        to a peer whose own state did not move.  Without ``peer_status_fn`` a
        node-wide state change counts as the candidate's change.
        """
        n_equal = max(1, Settings.GOSSIP_EXIT_ON_X_EQUAL_ROUNDS)
        last_status: Optional[str] = None
        equal_count = 0
        last_counted = 0.0
        last_sent: Dict[str, Tuple[Any, float]] = {}
        version = wakeup.version if wakeup is not None else 0

        def token(n: str) -> Any:
            if peer_status_fn is not None:
                return repr(peer_status_fn(n))
            return wakeup.version if wakeup is not None else version

        while True:
            t0 = time.monotonic()
            if early_stopping_fn() or self._terminate.is_set():
                logger.info(self._self_addr, "Stopping model gossip process.")
                return
            neis = get_candidates_fn()
            if not neis:
                logger.info(self._self_addr, "Gossip finished.")
                return
            # stall detection: identical snapshots at least one period apart
            status = repr(status_fn())
            if status != last_status:
                last_status, equal_count, last_counted = status, 1, t0
            elif t0 - last_counted >= period * 0.999:
                equal_count += 1
                last_counted = t0
                if equal_count >= n_equal:
                    logger.info(self._self_addr, f"Gossiping exited for {n_equal} equal rounds.")
                    return
            # choose fan-out among candidates that are due for a (re)send
            due = [
                n
                for n in neis
                if n not in last_sent or last_sent[n][0] != token(n) or (t0 - last_sent[n][1]) >= period * 0.999
            ]
            for nei in random.sample(due, min(Settings.GOSSIP_MODELS_PER_ROUND, len(due))):
                tok = token(nei)
                model = model_fn(nei)
                if model is None:
                    continue
                logger.debug(self._self_addr, f"Gossiping model to {nei}.")
                with logger.span(self._self_addr, "gossip_send", cmd=getattr(model, "cmd", "?"), to=nei):
                    self._client.send(nei, model, create_connection=create_connection)
                last_sent[nei] = (tok, time.monotonic())
            # wait for a state change or the rest of the period
            remaining = max(0.0, period - (time.monotonic() - t0))
            if wakeup is not None:
                version = wakeup.wait(version, remaining)
            elif remaining > 0:
                self._terminate.wait(remaining)
