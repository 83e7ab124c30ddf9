"""``models_ready`` (reference ``commands/models_ready_command.py:26-63``).

Records, for the sender, the round it reported ready (the highest seen, any
round up to the local one).  The reference records the *local* round instead
(quirk Q12): a neighbour's "ready for round r - 1" arriving at a node already in
round r then marks that neighbour up to date, the node's diffusion of its round-r
aggregate skips it, and the neighbour -- still waiting in round r for this node's
contribution -- hangs until AGGREGATION_TIMEOUT and aggregates without it (observed
in ``tests/test_gpu_fused_cnn.py::test_three_fused_peers_in_one_process``: one peer
finished round 1 three seconds before the others, which then ended round 2 with
different models).  Recording the reported round lets the diffusion reach it.
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
        if round <= r and (Settings.ASYNC_DIFFUSION or round >= r - 1):
            self.state.nei_status[source] = max(self.state.nei_status.get(source, -1), round)
            self.state.changed.bump()
        elif round > r:
            # a neighbour already past this node's round: it needs none of this
            # round's models (the partial-aggregate gossip stops offering them) and
            # none of this round's diffusion
            logger.debug(self.state.addr, f"Models ready from {source} for round {round} ahead of ours ({r}).")
            self.state.nei_status[source] = max(self.state.nei_status.get(source, -1), round)
            self.state.changed.bump()
        else:
            logger.error(self.state.addr, f"Models ready from {source} in a late round. Ignored. {round} != {r} / {r - 1}")
