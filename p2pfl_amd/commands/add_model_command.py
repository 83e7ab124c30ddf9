"""``add_model`` weights handler (reference ``commands/add_model_command.py:29-108``).

Feeds a partial or full aggregate into the aggregator and, if it was accepted,
announces the new contributor set with ``models_aggregated``.
"""

from __future__ import annotations

import time
from typing import Any, Callable, List, Optional

from p2pfl_amd.commands.command import Command
from p2pfl_amd.commands.models_agregated_command import ModelsAggregatedCommand
from p2pfl_amd.learning.exceptions import DecodingParamsError, ModelNotMatchingError
from p2pfl_amd.management.logger import logger
from p2pfl_amd.utils import finite


class AddModelCommand(Command):
    def __init__(self, state: Any, stop: Callable[[], None], aggregator: Any, comm_proto: Any) -> None:
        self.state = state
        self.stop = stop
        self.aggregator = aggregator
        self.communication_protocol = comm_proto

    @staticmethod
    def get_name() -> str:
        return "add_model"

    def precheck(self, source: str, round: int, contributors: List[str], weight: int) -> Optional[str]:
        """Why this payload would be ignored (None: it would be used), evaluated
        before the transfer (the receive path of the reference decoded every
        payload first: ``add_model_command.py:79-83``)."""
        if self.state.round is None or self.state.learner is None:
            return "learning not running"
        if round != self.state.round:
            return f"late round ({round} != {self.state.round})"
        if len(self.state.train_set) == 0:
            return "no train set"
        if not self.aggregator.would_accept(list(contributors)) and not self._probe_uncovered(list(contributors)):
            return "model not needed"
        return None

    def _probe_uncovered(self, contributors: List[str]) -> bool:
        """A waiting node is offered an aggregate that lacks train-set members it
        still believes alive (the sender already lost them; this node has not
        noticed yet -- e.g. no heartbeat timeout so far).  Probe those members
        right away: an unreachable one is dropped from the neighbour table and
        marked lost, and the offer is re-evaluated.  True if it is acceptable now.

        Without this, the diffusion loop of the sender can give up (stall exit)
        before this node's heartbeat timeout fires, and the node then waits for
        AGGREGATION_TIMEOUT.
        """
        missing = self.aggregator.uncovered(contributors)
        if not missing:
            return False
        proto = self.communication_protocol
        known = proto.get_neighbors(only_direct=False)
        gone = [m for m in missing if m not in known]
        for m in missing:
            if m in known:
                # a failed send removes the neighbour; the node's neighbour
                # listener then marks it lost in the aggregator
                proto.send(m, proto.build_msg("beat", [str(time.time())]), create_connection=True)
                if m not in proto.get_neighbors(only_direct=False):
                    gone.append(m)
        if gone:
            self.aggregator.mark_lost(gone)
        return self.aggregator.would_accept(contributors)

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
            raise ValueError("Weights, contributors and weight are required")
        if self.state.round is None:
            logger.debug(self.state.addr, "Tried to add a model while learning is not running")
            return
        if round != self.state.round:
            logger.debug(self.state.addr, f"Model reception in a late round ({round} != {self.state.round}).")
            return
        if len(self.state.train_set) == 0:
            logger.error(self.state.addr, "Model Reception when there is no trainset")
            return
        learner = self.state.learner
        if learner is None:
            return
        try:
            # cheap pre-check: skip decoding models the aggregator would reject
            if not self.aggregator.would_accept(list(contributors)) and not self._probe_uncovered(list(contributors)):
                logger.debug(self.state.addr, f"Model from {contributors} not needed; skipped decode.")
                return
            params = learner.decode_parameters(weights)
            finite.check(self.state.addr, "received model", params, source=source, contributors=list(contributors),
                         round=round)
            models_added = self.aggregator.add_model(params, list(contributors), weight)
            if not models_added and self._probe_uncovered(list(contributors)):
                models_added = self.aggregator.add_model(params, list(contributors), weight)
            if models_added:
                self.state.changed.bump()
                # the report carries the round of the models it lists: the add that
                # completes the aggregation can let the learning thread move on at once,
                # and a report stamped with the NEW round is ignored by every peer still
                # in this one -- they kept offering this node models until their gossip
                # loop's equal-rounds exit (~GOSSIP_EXIT_ON_X_EQUAL_ROUNDS periods, 9 s
                # stalls of the 8-peer bench_node rounds)
                self.communication_protocol.broadcast(
                    self.communication_protocol.build_msg(ModelsAggregatedCommand.get_name(), models_added, round=round)
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
