"""``stop_learning`` (reference ``commands/stop_learning_command.py:27-61``)."""

from __future__ import annotations

from typing import Any

from p2pfl_amd.commands.command import Command
from p2pfl_amd.management.logger import logger


class StopLearningCommand(Command):
    def __init__(self, state: Any, aggregator: Any) -> None:
        self.state = state
        self.aggregator = aggregator

    @staticmethod
    def get_name() -> str:
        return "stop_learning"

    def execute(self, source: str, round: int, *args, **kwargs) -> None:
        logger.info(self.state.addr, "Stopping learning")
        learner = self.state.learner
        if learner is not None:
            learner.interrupt_fit()
        self.state.learner = None
        self.aggregator.clear()
        self.state.clear()
        logger.experiment_finished(self.state.addr)
