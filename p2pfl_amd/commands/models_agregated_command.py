"""``models_aggregated c1 c2 ...`` (reference ``commands/models_agregated_command.py:26-56``)."""

from __future__ import annotations

from typing import Any

from p2pfl_amd.commands.command import Command
from p2pfl_amd.management.logger import logger


class ModelsAggregatedCommand(Command):
    def __init__(self, state: Any) -> None:
        self.state = state

    @staticmethod
    def get_name() -> str:
        return "models_aggregated"

    def execute(self, source: str, round: int, *args, **kwargs) -> None:
        if round == self.state.round:
            self.state.models_aggregated[source] = list(args)
            self.state.changed.bump()
        else:
            logger.debug(
                self.state.addr,
                f"Models Aggregated message from {source} in a late round. Ignored. {round} != {self.state.round}",
            )
