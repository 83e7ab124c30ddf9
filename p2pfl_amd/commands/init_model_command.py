"""``init_model`` weights handler (reference ``commands/init_model_command.py:29-117``).

Loads the initiator's weights once per experiment, then announces
``model_initialized``.  A payload that cannot be decoded or does not match the
local model stops the node, like the reference (the reference itself notes this
enables denial of service; kept for behavioural parity and covered by
``test_wrong_model``).
"""

from __future__ import annotations

from typing import Any, Callable, List, Optional

from p2pfl_amd.commands.command import Command
from p2pfl_amd.commands.model_initialized_command import ModelInitializedCommand
from p2pfl_amd.learning.exceptions import DecodingParamsError, ModelNotMatchingError
from p2pfl_amd.management.logger import logger


class InitModelCommand(Command):
    def __init__(self, state: Any, stop: Callable[[], None], aggregator: Any, comm_proto: Any) -> None:
        self.state = state
        self.stop = stop
        self.aggregator = aggregator
        self.communication_protocol = comm_proto

    @staticmethod
    def get_name() -> str:
        return "init_model"

    def precheck(self, source: str, round: int, contributors: List[str], weight: int) -> Optional[str]:
        """Why this payload would be ignored (None: it would be used) -- lets a
        data-plane transport decline a transfer before any byte moves."""
        if self.state.learner is None:
            return "learner not ready"
        if round != self.state.round:
            return f"late round ({round} != {self.state.round})"
        if self.state.model_initialized.is_set():
            return "model already initialized"
        return None

    def execute(
        self,
        source: str,
        round: int,
        weights: Any = None,
        contributors: Optional[List[str]] = None,
        weight: Optional[int] = None,
        **kwargs,
    ) -> None:
        if weights is None or contributors is None or weight is None:
            logger.error(self.state.addr, "Invalid message")
            return
        learner = self.state.learner
        if learner is None:
            logger.debug(self.state.addr, "Tried to add a model while learning is not running")
            return
        if round != self.state.round:
            logger.debug(self.state.addr, f"Model reception in a late round ({round} != {self.state.round}).")
            return
        if self.state.model_initialized.is_set():
            logger.debug(self.state.addr, "Model initialization message when the model is already initialized. Ignored.")
            return
        try:
            learner.set_parameters(learner.decode_parameters(weights))
            self.state.model_initialized.set()
            self.state.changed.bump()
            logger.info(self.state.addr, "Model Weights Initialized")
            self.communication_protocol.broadcast(
                self.communication_protocol.build_msg(ModelInitializedCommand.get_name())
            )
        except DecodingParamsError:
            logger.error(self.state.addr, "Error decoding parameters.")
            self.stop()
        except ModelNotMatchingError:
            logger.error(self.state.addr, "Models not matching.")
            self.stop()
        except Exception as e:
            logger.error(self.state.addr, f"Unknown error adding model: {e}")
            self.stop()
