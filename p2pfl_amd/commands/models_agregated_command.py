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
            # a node's set of aggregated models only grows within a round, but its
            # reports travel on concurrent sender threads (two models added at once
            # broadcast 7/8 and 8/8 side by side): a stale report overwriting a newer
            # one made peers push models the node already held until their
            # equal-rounds exit (the reference assigns: models_agregated_command.py:49)
            prev = self.state.models_aggregated.get(source, [])
            self.state.models_aggregated[source] = prev + [c for c in args if c not in prev]
            self.state.changed.bump()
        else:
            logger.debug(
                self.state.addr,
                f"Models Aggregated message from {source} in a late round. Ignored. {round} != {self.state.round}",
            )
