"""WaitAggregatedModelsStage (reference ``stages/base_node/wait_agg_models_stage.py:31-49``)."""

from __future__ import annotations

from typing import Any, Optional, Type

from p2pfl_amd.management.logger import logger
from p2pfl_amd.stages.stage import Stage
from p2pfl_amd.stages.stage_factory import StageFactory


class WaitAggregatedModelsStage(Stage):
    @staticmethod
    def name() -> str:
        return "WaitAggregatedModelsStage"

    @staticmethod
    def execute(
        state: Any = None, aggregator: Any = None, communication_protocol: Any = None, **kwargs
    ) -> Optional[Type[Stage]]:
        if state is None or aggregator is None:
            raise Exception("Invalid parameters on WaitAggregatedModelsStage.")
        logger.info(state.addr, "Waiting aggregation.")
        aggregator.set_waiting_aggregated_model(state.train_set)
        if communication_protocol is not None:
            from p2pfl_amd.stages.base_node.common import mark_dead_train_set_members

            mark_dead_train_set_members(state, communication_protocol, aggregator)
        return StageFactory.get_stage("GossipModelStage")
