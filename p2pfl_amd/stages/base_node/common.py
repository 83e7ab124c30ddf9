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
    logger.info(state.addr, "Evaluating...")
    if state.learner is None:
        raise Exception("Learner not initialized.")
    results = state.learner.evaluate()
    logger.info(state.addr, f"Evaluated. Results: {results}")
    if results:
        flat = [str(x) for kv in results.items() for x in kv]
        protocol.broadcast(protocol.build_msg(MetricsCommand.get_name(), flat, round=state.round))
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
