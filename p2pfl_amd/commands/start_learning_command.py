"""``start_learning <rounds> <epochs>`` (reference ``commands/start_learning_command.py:26-60``)."""

from __future__ import annotations

from typing import Callable, Optional

from p2pfl_amd.commands.command import Command


class StartLearningCommand(Command):
    def __init__(self, start_learning_fn: Callable[[int, int], None]) -> None:
        self._learning_fn = start_learning_fn

    @staticmethod
    def get_name() -> str:
        return "start_learning"

    def execute(
        self, source: str, round: int, learning_rounds: Optional[str] = None, learning_epochs: Optional[str] = None, *a, **kw
    ) -> None:
        if learning_rounds is None or learning_epochs is None:
            raise ValueError("Learning rounds and epochs are required")
        self._learning_fn(int(learning_rounds), int(learning_epochs))
