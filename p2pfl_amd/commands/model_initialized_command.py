"""``model_initialized`` (reference ``commands/model_initialized_command.py:25-48``)."""

from __future__ import annotations

from typing import Any

from p2pfl_amd.commands.command import Command


class ModelInitializedCommand(Command):
    def __init__(self, state: Any) -> None:
        self.state = state

    @staticmethod
    def get_name() -> str:
        return "model_initialized"

    def execute(self, source: str, round: int, *args, **kwargs) -> None:
        self.state.nei_status[source] = -1
        self.state.changed.bump()
