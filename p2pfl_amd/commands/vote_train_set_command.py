"""``vote_train_set n1 w1 n2 w2 ...`` (reference ``commands/vote_train_set_command.py:28-74``).

Votes are accepted for the current round or the next one (nodes run
asynchronously); the waiting vote stage is woken through a condition variable.
"""

from __future__ import annotations

from typing import Any

from p2pfl_amd.commands.command import Command
from p2pfl_amd.management.logger import logger


class VoteTrainSetCommand(Command):
    def __init__(self, state: Any) -> None:
        self.state = state

    @staticmethod
    def get_name() -> str:
        return "vote_train_set"

    def execute(self, source: str, round: int, *args, **kwargs) -> None:
        r = self.state.round
        if r is None:
            logger.error(self.state.addr, "Vote received when learning is not running")
            return
        if round not in (r, r + 1):
            logger.error(self.state.addr, f"Vote received in a late round. Ignored. {round} != {r} / {r + 1}")
            return
        votes = {args[i]: int(args[i + 1]) for i in range(0, len(args) - 1, 2)}
        with self.state.train_set_votes_lock:
            self.state.train_set_votes[source] = votes
        self.state.notify_vote()
