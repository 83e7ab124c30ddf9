"""``models_ready`` (reference ``commands/models_ready_command.py:26-63``).

Accepts the current or the previous round and records the *local* round for
the sender (reference quirk Q12, preserved).  With
``Settings.ASYNC_DIFFUSION`` a node may already train round r+1 when a
neighbour's "ready for round r" arrives; recording the local round there
would mark the neighbour as up to date and stop the diffusion it still
needs, so that mode records the round the neighbour actually reported (the
highest seen, any round up to the local one).
"""

from __future__ import annotations

from typing import Any

from p2pfl_amd.commands.command import Command
from p2pfl_amd.management.logger import logger
from p2pfl_amd.settings import Settings


class ModelsReadyCommand(Command):
    def __init__(self, state: Any) -> None:
        self.state = state

    @staticmethod
    def get_name() -> str:
        return "models_ready"

    def execute(self, source: str, round: int, *args, **kwargs) -> None:
        r = self.state.round
        if r is None:
            logger.warning(self.state.addr, "Models ready received when learning is not running")
            return
        if Settings.ASYNC_DIFFUSION:
            if round <= r:
                self.state.nei_status[source] = max(self.state.nei_status.get(source, -1), round)
                self.state.changed.bump()
            else:
                logger.debug(self.state.addr, f"Models ready from {source} for round {round} ahead of ours ({r}).")
            return
        if round in (r - 1, r):
            self.state.nei_status[source] = r
            self.state.changed.bump()
        else:
            logger.error(self.state.addr, f"Models ready from {source} in a late round. Ignored. {round} != {r} / {r - 1}")
