"""Per-step metric adapter for learners (reference ``lightning_logger.py:29-68``).

The reference plugs a Lightning ``Logger`` into the Trainer so per-batch
training metrics land in the p2pfl logger's local storage.  There is no
Lightning here; :class:`FederatedLogger` keeps the same small API
(``name``, ``version``, ``log_hyperparams``, ``log_metrics(metrics, step)``)
so learner code written against the reference keeps working, and
``TorchLearner`` / ``FusedCNNLearner`` report through the same path.
"""

from __future__ import annotations

from typing import Any, Dict, Optional

from p2pfl_amd.management.logger import logger


class FederatedLogger:
    def __init__(self, node_name: str) -> None:
        self.self_name = node_name

    @property
    def name(self) -> str:
        return "p2pfl"

    @property
    def version(self) -> str:
        return "0.3.0-amd"

    def log_hyperparams(self, params: Dict[str, Any]) -> None:
        """Hyper-parameters are not stored (same as the reference)."""

    def log_metrics(self, metrics: Dict[str, float], step: Optional[int]) -> None:
        for k, v in metrics.items():
            logger.log_metric(self.self_name, k, float(v), step=step)

    def save(self) -> None:
        """Nothing to flush (same as the reference)."""

    def finalize(self, status: str) -> None:
        """Nothing to close (same as the reference)."""
