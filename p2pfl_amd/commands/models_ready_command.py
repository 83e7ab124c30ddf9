"""``models_ready`` (reference ``commands/models_ready_command.py:26-63``).

Accepts the current or the previous round and records the *local* round for
the sender (reference quirk Q12, preserved).
"""

from __future__ import annotations

from typing import Any

from p2pfl_amd.commands.command import Command
from p2pfl_amd.management.logger import logger


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
        if round in (r - 1, r):
            self.state.nei_status[source] = r
            self.state.changed.bump()
        else:
            logger.error(self.state.addr, f"Models ready from {source} in a late round. Ignored. {round} != {r} / {r - 1}")
