"""TrainStage (reference ``stages/base_node/train_stage.py:35-184``).

Evaluate -> fit -> add the own model to the aggregator -> push partial
aggregates to train-set peers until every train-set model has been collected.
Non-members of the train set (which the reference also routed here from round
2 on, only to have their model rejected: quirk Q3) go straight to waiting for
the full aggregate.
"""

from __future__ import annotations

from typing import Any, List, Optional, Type

from p2pfl_amd.commands.add_model_command import AddModelCommand
from p2pfl_amd.commands.models_agregated_command import ModelsAggregatedCommand
from p2pfl_amd.management.logger import logger
from p2pfl_amd.stages.base_node.common import evaluate_and_share, model_payload, mark_dead_train_set_members
from p2pfl_amd.stages.stage import Stage
from p2pfl_amd.stages.stage_factory import StageFactory


class TrainStage(Stage):
    @staticmethod
    def name() -> str:
        return "TrainStage"

    @staticmethod
    def execute(
        state: Any = None,
        communication_protocol: Any = None,
        aggregator: Any = None,
        early_stopping_fn: Any = None,
        **kwargs,
    ) -> Optional[Type[Stage]]:
        if state is None or communication_protocol is None or aggregator is None or early_stopping_fn is None:
            raise Exception("Invalid parameters on TrainStage.")
        if state.addr not in state.train_set:
            return StageFactory.get_stage("WaitAggregatedModelsStage")
        if not early_stopping_fn():
            aggregator.set_nodes_to_aggregate(state.train_set)
            mark_dead_train_set_members(state, communication_protocol, aggregator)
        if not early_stopping_fn():
            evaluate_and_share(state, communication_protocol)
        if not early_stopping_fn():
            logger.info(state.addr, "Training...")
            with logger.span(state.addr, "fit", round=state.round):
                state.learner.fit()
        if not early_stopping_fn():
            learner = state.learner
            models_added = aggregator.add_model(learner.get_parameters(), [state.addr], learner.get_num_samples()[0])
            state.changed.bump()
            communication_protocol.broadcast(
                communication_protocol.build_msg(ModelsAggregatedCommand.get_name(), models_added, round=state.round)
            )
            TrainStage._gossip_model_aggregation(state, communication_protocol, aggregator)
        return StageFactory.get_stage("GossipModelStage")

    @staticmethod
    def _gossip_model_aggregation(state: Any, protocol: Any, aggregator: Any) -> None:
        def peer_has(n: str) -> List[str]:
            return state.models_aggregated.get(n, [])

        def candidates() -> List[str]:
            # A train-set peer is a candidate while it lacks some of the models
            # this node holds (per its models_aggregated reports).  The
            # reference (train_stage.py:134-139) used "its model is not in my
            # aggregate", which stops pushing as soon as the peer's model
            # arrived here even if the peer never received this node's model
            # (its own comment flags the hazard): on a partial topology that
            # leaves peers waiting for AGGREGATION_TIMEOUT.
            have = set(aggregator.get_aggregated_models())
            return [
                n
                for n in protocol.get_neighbors(only_direct=False)
                if n in state.train_set and n != state.addr and (have - set(peer_has(n)))
            ]

        def status() -> Any:
            return [(n, peer_has(n)) for n in protocol.get_neighbors(only_direct=False) if n in state.train_set]

        def model_fn(node: str) -> Any:
            model, contributors, weight = aggregator.get_partial_aggregation(peer_has(node))
            if model is None or state.round is None or state.learner is None:
                return None
            return protocol.build_weights(
                AddModelCommand.get_name(), state.round, model_payload(state, protocol, model), contributors, weight
            )

        protocol.gossip_weights(
            lambda: state.round is None,
            candidates,
            status,
            model_fn,
            create_connection=True,
            wakeup=state.changed,
            # a re-send is due when the peer's report moved OR this node's own
            # aggregate grew (a richer partial aggregate goes out at once
            # instead of waiting a GOSSIP_MODELS_PERIOD per hop)
            peer_status_fn=lambda n: (peer_has(n), sorted(aggregator.get_aggregated_models())),
        )
