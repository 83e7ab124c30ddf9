"""``metrics k1 v1 k2 v2 ...`` (reference ``commands/metrics_command.py:26-55``).

Remote metrics are stored under the sender's name even if the sender is not
registered in this process (reference quirk Q7 fixed in the logger).
"""

from __future__ import annotations

from typing import Any

from p2pfl_amd.commands.command import Command
from p2pfl_amd.management.logger import logger


class MetricsCommand(Command):
    def __init__(self, state: Any) -> None:
        self.state = state

    @staticmethod
    def get_name() -> str:
        return "metrics"

    def execute(self, source: str, round: int, *args, **kwargs) -> None:
        logger.info(self.state.addr, f"Metrics received from {source}")
        exp = self.state.actual_exp_name or "experiment"
        for i in range(0, len(args) - 1, 2):
            logger.log_metric(source, args[i], float(args[i + 1]), round=round, exp=exp)
