"""Message handlers (command pattern); the names are wire-visible."""

from p2pfl_amd.commands.add_model_command import AddModelCommand
from p2pfl_amd.commands.command import Command
from p2pfl_amd.commands.heartbeat_command import HeartbeatCommand
from p2pfl_amd.commands.init_model_command import InitModelCommand
from p2pfl_amd.commands.metrics_command import MetricsCommand
from p2pfl_amd.commands.model_initialized_command import ModelInitializedCommand
from p2pfl_amd.commands.models_agregated_command import ModelsAggregatedCommand
from p2pfl_amd.commands.models_ready_command import ModelsReadyCommand
from p2pfl_amd.commands.start_learning_command import StartLearningCommand
from p2pfl_amd.commands.stop_learning_command import StopLearningCommand
from p2pfl_amd.commands.vote_train_set_command import VoteTrainSetCommand

__all__ = [
    "Command",
    "AddModelCommand",
    "HeartbeatCommand",
    "InitModelCommand",
    "MetricsCommand",
    "ModelInitializedCommand",
    "ModelsAggregatedCommand",
    "ModelsReadyCommand",
    "StartLearningCommand",
    "StopLearningCommand",
    "VoteTrainSetCommand",
]
