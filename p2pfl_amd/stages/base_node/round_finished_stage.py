"""RoundFinishedStage (reference ``stages/base_node/round_finished_stage.py:34-97``)."""

from __future__ import annotations

from typing import Any, Optional, Type

from p2pfl_amd.management.logger import logger
from p2pfl_amd.stages.base_node.common import evaluate_and_share
from p2pfl_amd.stages.stage import Stage
from p2pfl_amd.stages.stage_factory import StageFactory


class RoundFinishedStage(Stage):
    @staticmethod
    def name() -> str:
        return "RoundFinishedStage"

    @staticmethod
    def execute(
        state: Any = None,
        communication_protocol: Any = None,
        aggregator: Any = None,
        early_stopping_fn: Any = None,
        **kwargs,
    ) -> Optional[Type[Stage]]:
        if state is None or communication_protocol is None or aggregator is None or early_stopping_fn is None:
            raise Exception("Invalid parameters on RoundFinishedStage.")
        if early_stopping_fn():
            logger.info(state.addr, "Early stopping.")
            return None
        aggregator.clear()
        state.increase_round()
        logger.round_finished(state.addr)
        logger.info(state.addr, f"Round {state.round} of {state.total_rounds} finished.")
        if state.round is None or state.total_rounds is None:
            raise Exception("Round or total rounds not set.")
        if state.round < state.total_rounds:
            return StageFactory.get_stage("TrainStage")
        evaluate_and_share(state, communication_protocol)
        # experiment over: reset per-experiment peer bookkeeping so a new
        # experiment re-gossips the initial model (the reference kept stale
        # nei_status entries and could stall a second experiment)
        state.nei_status = {}
        state.train_set = []
        state.model_initialized.clear()
        state.clear()
        logger.info(state.addr, "Training finished!!.")
        return None
