"""Round state machine: StartLearning -> VoteTrainSet -> Train | WaitAggregatedModels -> GossipModel -> RoundFinished."""

from p2pfl_amd.stages.stage import Stage
from p2pfl_amd.stages.stage_factory import StageFactory
from p2pfl_amd.stages.workflows import LearningWorkflow, StageWorkflow

__all__ = ["Stage", "StageFactory", "LearningWorkflow", "StageWorkflow"]
