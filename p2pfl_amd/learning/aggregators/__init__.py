"""Aggregation strategies."""

from p2pfl_amd.learning.aggregators.aggregator import Aggregator, NoModelsToAggregateError
from p2pfl_amd.learning.aggregators.fedavg import FedAvg

__all__ = ["Aggregator", "NoModelsToAggregateError", "FedAvg"]
