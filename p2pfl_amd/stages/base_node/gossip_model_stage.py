"""GossipModelStage (reference ``stages/base_node/gossip_model_stage.py:34-132``).

Wait for the aggregation, load it, announce ``models_ready``, then diffuse the
full model to direct neighbours that are still behind this round.
"""

from __future__ import annotations

from typing import Any, List, Optional, Type

from p2pfl_amd.commands.add_model_command import AddModelCommand
from p2pfl_amd.commands.models_ready_command import ModelsReadyCommand
from p2pfl_amd.management.logger import logger
from p2pfl_amd.stages.base_node.common import model_payload
from p2pfl_amd.stages.stage import Stage
from p2pfl_amd.stages.stage_factory import StageFactory


class GossipModelStage(Stage):
    @staticmethod
    def name() -> str:
        return "GossipModelStage"

    @staticmethod
    def execute(
        state: Any = None,
        communication_protocol: Any = None,
        aggregator: Any = None,
        early_stopping_fn: Any = None,
        **kwargs,
    ) -> Optional[Type[Stage]]:
        if state is None or aggregator is None or early_stopping_fn is None or communication_protocol is None:
            raise Exception("Invalid parameters on GossipModelStage.")
        if not early_stopping_fn():
            GossipModelStage._wait_aggregated_model(state, communication_protocol, aggregator)
        if not early_stopping_fn():
            GossipModelStage._gossip_model_diffusion(state, communication_protocol, aggregator)
        return StageFactory.get_stage("RoundFinishedStage")

    @staticmethod
    def _wait_aggregated_model(state: Any, protocol: Any, aggregator: Any) -> None:
        with logger.span(state.addr, "wait_aggregation", round=state.round):
            params = aggregator.wait_and_get_aggregation()
        if state.round is None:
            return
        if params is not None:
            if state.learner is None:
                raise Exception("Learner not initialized")
            state.learner.set_parameters(params)
        else:
            logger.warning(state.addr, "No aggregated model available; continuing with the local model.")
        logger.debug(state.addr, f"Broadcast aggregation done for round {state.round}")
        protocol.broadcast(protocol.build_msg(ModelsReadyCommand.get_name(), [], round=state.round))

    @staticmethod
    def _gossip_model_diffusion(state: Any, protocol: Any, aggregator: Any) -> None:
        logger.info(state.addr, "Gossiping aggregated model.")
        fixed_round = state.round
        if fixed_round is None:
            return

        def candidates() -> List[str]:
            return [
                n
                for n in protocol.get_neighbors(only_direct=True)
                if n in state.nei_status and state.nei_status[n] < fixed_round
            ]

        def model_fn(_: str) -> Any:
            if state.learner is None or state.round is None:
                return None
            return protocol.build_weights(
                AddModelCommand.get_name(),
                state.round,
                model_payload(state, protocol),
                aggregator.get_aggregated_models(),
                1,
            )

        protocol.gossip_weights(
            lambda: state.round is None,
            candidates,
            candidates,
            model_fn,
            wakeup=state.changed,
            peer_status_fn=lambda n: state.nei_status.get(n),
        )
