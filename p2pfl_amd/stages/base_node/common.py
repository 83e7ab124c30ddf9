"""Helpers shared by stages."""

from __future__ import annotations

import threading
import time
from typing import Any, Callable, Dict, List, Optional, Set, Tuple

from p2pfl_amd.commands.metrics_command import MetricsCommand
from p2pfl_amd.management.logger import logger
from p2pfl_amd.settings import Settings


def model_payload(state: Any, protocol: Any, params: Optional[Any] = None) -> Any:
    """Encode a model for the wire, or snapshot it on the device if the transport allows."""
    learner = state.learner
    if learner is None:
        raise Exception("Learner not initialized.")
    if getattr(protocol, "supports_device_payloads", False):
        return learner.snapshot_parameters(params)
    return learner.encode_parameters(params)


def evaluate_and_share(state: Any, protocol: Any) -> Dict[str, float]:
    """Evaluate the local model and broadcast the metrics (reference
    ``train_stage.py:95-112``).  With an asynchronous learner the pass is only
    enqueued here; the metrics go out from its completion thread when they land
    (returns ``{}``), so the round does not wait for the test pass."""
    logger.info(state.addr, "Evaluating...")
    learner = state.learner
    if learner is None:
        raise Exception("Learner not initialized.")
    rnd = state.round

    def share(results: Dict[str, float]) -> None:
        logger.info(state.addr, f"Evaluated. Results: {results}")
        if results:
            flat = [str(x) for kv in results.items() for x in kv]
            try:
                protocol.broadcast(protocol.build_msg(MetricsCommand.get_name(), flat, round=rnd))
            except Exception as e:  # the node may have stopped meanwhile
                logger.debug(state.addr, f"metrics broadcast skipped: {e}")

    if learner.evaluate_async(share):
        return {}
    results = learner.evaluate()
    share(results)
    return results


def mark_dead_train_set_members(state: Any, protocol: Any, aggregator: Any) -> None:
    """Tell the aggregator which train-set members are no longer in the neighbour table.

    The train set is voted once per experiment (reference
    ``round_finished_stage.py:69-70``), so a member that died in an earlier
    round is still expected in later ones; without this every later round
    would wait ``AGGREGATION_TIMEOUT`` for it.  A "lost" member whose model
    still arrives is accepted (the aggregator un-marks it).
    """
    live = set(protocol.get_neighbors(only_direct=False)) | {state.addr}
    lost = [n for n in state.train_set if n not in live]
    if lost:
        aggregator.mark_lost(lost)


def relay_grace(state: Any = None, protocol: Any = None) -> float:
    """``Settings.GOSSIP_RELAY_GRACE`` (None: a quarter of ``GOSSIP_MODELS_PERIOD``),
    or 0 (relay at once) unless every train-set member is a direct neighbour --
    only then can the origins be expected to deliver their own models."""
    g = Settings.GOSSIP_RELAY_GRACE
    g = float(0.25 * Settings.GOSSIP_MODELS_PERIOD if g is None else g)
    if g > 0 and state is not None and protocol is not None:
        direct = set(protocol.get_neighbors(only_direct=True)) | {state.addr}
        if not set(getattr(state, "train_set", ()) or ()) <= direct:
            return 0.0
    return g


class ReportClock:
    """When each peer's status report last changed (a report that has not
    moved for the relay grace means the origin of what it lacks is not getting
    through, so this node relays)."""

    def __init__(self, report_fn: Callable[[str], Any]) -> None:
        self._fn = report_fn
        self._seen: Dict[str, Tuple[str, float]] = {}

    def get(self, peer: str) -> Tuple[str, float]:
        """(the report as a token, monotonic time it last changed)."""
        rep = repr(self._fn(peer))
        prev = self._seen.get(peer)
        if prev is None or prev[0] != rep:
            prev = self._seen[peer] = (rep, time.monotonic())
        return prev


class DeliveryLedger:
    """What one gossip stage offered each peer and what became of it.

    Exactly-once model delivery (new; the reference re-pushes every period to
    every candidate: ``gossiper.py:228-239``): a contribution that is on its
    way to a peer (the xGMI plane reports ``pending`` at the proposal,
    ``delivered`` after the transfer) or already delivered is not offered
    again; a ``declined`` one (e.g. the peer was still in the previous round)
    is.  Transports without delivery feedback keep the reference behaviour: an
    offer counts until the peer's status report changes or one
    ``GOSSIP_MODELS_PERIOD`` passed (a push the receiver ignored -- e.g. it was
    still in the previous round -- is sent again, as the reference re-sends
    every period).  A proposal with no answer within ``expiry`` seconds no
    longer counts (the plane lost it).
    """

    def __init__(self, expiry: float) -> None:
        self.expiry = expiry
        self.resend = float(Settings.GOSSIP_MODELS_PERIOD)
        self._lock = threading.Lock()
        self._rec: Dict[str, Dict[frozenset, List[Any]]] = {}

    def attach(self, peer: str, msg: Any, token: str) -> Any:
        entry: List[Any] = ["sent", token, time.monotonic()]
        with self._lock:
            self._rec.setdefault(peer, {})[frozenset(getattr(msg, "contributors", ()) or ("?",))] = entry

        def on_result(res: str) -> None:
            with self._lock:
                entry[0] = res if res in ("pending", "delivered") else "declined"
                entry[2] = time.monotonic()

        try:
            msg.on_result = on_result
        except AttributeError:  # a custom protocol's message type: no feedback
            pass
        return msg

    def covered(self, peer: str, token: str) -> Set[str]:
        """Contributors offered to ``peer`` that count as on their way."""
        now = time.monotonic()
        out: Set[str] = set()
        with self._lock:
            for key, (st, tok, t) in self._rec.get(peer, {}).items():
                if (st == "delivered" or (st == "pending" and now - t < self.expiry)
                        or (st == "sent" and tok == token and now - t < self.resend)):
                    out |= key
        return out
