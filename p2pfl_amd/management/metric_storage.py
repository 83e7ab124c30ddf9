"""In-memory metric stores.

Shapes are kept identical to the reference (``metric_storage.py:24-27``,
``:153``) because examples and user code index them directly:

* local  : experiment -> round -> node -> metric -> [(step, value), ...]
* global : experiment -> node -> metric -> [(round, value), ...]   (first value per round wins)
"""

from __future__ import annotations

import threading
from typing import Dict, List, Tuple, Union

MetricsType = Dict[str, List[Tuple[int, float]]]
NodeLogsType = Dict[str, MetricsType]
RoundLogsType = Dict[int, NodeLogsType]
LocalLogsType = Dict[str, RoundLogsType]
GlobalLogsType = Dict[str, NodeLogsType]

Number = Union[int, float]


class LocalMetricStorage:
    """Per-step training metrics of every node, by experiment and round."""

    def __init__(self) -> None:
        self.exp_dicts: LocalLogsType = {}
        self.lock = threading.Lock()

    def add_log(self, exp_name: str, round: int, metric: str, node: str, val: Number, step: int) -> None:
        with self.lock:
            series = (
                self.exp_dicts.setdefault(exp_name, {})
                .setdefault(round, {})
                .setdefault(node, {})
                .setdefault(metric, [])
            )
            series.append((step, val))

    def get_all_logs(self) -> LocalLogsType:
        return self.exp_dicts

    def get_experiment_logs(self, exp: str) -> RoundLogsType:
        return self.exp_dicts[exp]

    def get_experiment_round_logs(self, exp: str, round: int) -> NodeLogsType:
        return self.exp_dicts[exp][round]

    def get_experiment_round_node_logs(self, exp: str, round: int, node: str) -> MetricsType:
        return self.exp_dicts[exp][round][node]


class GlobalMetricStorage:
    """Per-round evaluation metrics of every node (own and received)."""

    def __init__(self) -> None:
        self.exp_dicts: GlobalLogsType = {}
        self.lock = threading.Lock()

    def add_log(self, exp_name: str, round: int, metric: str, node: str, val: Number) -> None:
        with self.lock:
            series = self.exp_dicts.setdefault(exp_name, {}).setdefault(node, {}).setdefault(metric, [])
            # keep only the first value reported for a round (reference dedupe)
            if all(r != round for r, _ in series):
                series.append((round, val))

    def get_all_logs(self) -> GlobalLogsType:
        return self.exp_dicts

    def get_experiment_logs(self, exp: str) -> NodeLogsType:
        return self.exp_dicts[exp]

    def get_experiment_node_logs(self, exp: str, node: str) -> MetricsType:
        return self.exp_dicts[exp][node]
