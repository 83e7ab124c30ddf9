"""Helpers shared by stages."""

from __future__ import annotations

from typing import Any, Dict, Optional

from p2pfl_amd.commands.metrics_command import MetricsCommand
from p2pfl_amd.management.logger import logger


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
