"""Stage lookup by name (reference ``stages/stage_factory.py:26-59``); lazy imports avoid cycles."""

from __future__ import annotations

import importlib
from typing import Type

from p2pfl_amd.stages.stage import Stage

_STAGES = {
    "StartLearningStage": "p2pfl_amd.stages.base_node.start_learning_stage",
    "VoteTrainSetStage": "p2pfl_amd.stages.base_node.vote_train_set_stage",
    "TrainStage": "p2pfl_amd.stages.base_node.train_stage",
    "WaitAggregatedModelsStage": "p2pfl_amd.stages.base_node.wait_agg_models_stage",
    "GossipModelStage": "p2pfl_amd.stages.base_node.gossip_model_stage",
    "RoundFinishedStage": "p2pfl_amd.stages.base_node.round_finished_stage",
}


class StageFactory:
    @staticmethod
    def get_stage(stage_name: str) -> Type[Stage]:
        mod = _STAGES.get(stage_name)
        if mod is None:
            raise Exception("Invalid stage name.")
        return getattr(importlib.import_module(mod), stage_name)
