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
