"""Simulation / test helpers (reference ``p2pfl/utils.py:37-138``)."""

from __future__ import annotations

import time
from typing import Any, List

import numpy as np
import torch

from p2pfl_amd.settings import Settings


def set_test_settings() -> None:
    """Shrink timers for tests (same values as the reference)."""
    Settings.GRPC_TIMEOUT = 0.5
    Settings.HEARTBEAT_PERIOD = 0.5
    Settings.HEARTBEAT_TIMEOUT = 2
    Settings.GOSSIP_PERIOD = 0
    Settings.TTL = 10
    Settings.GOSSIP_MESSAGES_PER_PERIOD = 100
    Settings.AMOUNT_LAST_MESSAGES_SAVED = 100
    Settings.GOSSIP_MODELS_PERIOD = 1
    Settings.GOSSIP_MODELS_PER_ROUND = 4
    Settings.GOSSIP_EXIT_ON_X_EQUAL_ROUNDS = 4
    Settings.TRAIN_SET_SIZE = 4
    Settings.VOTE_TIMEOUT = 60
    Settings.AGGREGATION_TIMEOUT = 60
    Settings.WAIT_HEARTBEATS_CONVERGENCE = 0.2 * Settings.HEARTBEAT_TIMEOUT
    Settings.LOG_LEVEL = "DEBUG"


def wait_convergence(nodes: List[Any], n_neis: int, wait: float = 5, only_direct: bool = False) -> None:
    """Block until every node sees ``n_neis`` neighbours; AssertionError after ``wait`` s."""
    deadline = time.monotonic() + wait
    while True:
        if all(len(n.get_neighbors(only_direct=only_direct)) == n_neis for n in nodes):
            return
        if time.monotonic() > deadline:
            raise AssertionError(
                f"no convergence to {n_neis} neighbours: {[len(n.get_neighbors(only_direct=only_direct)) for n in nodes]}"
            )
        time.sleep(0.05)


def full_connection(node: Any, nodes: List[Any]) -> None:
    for n in nodes:
        node.connect(n.addr)


def wait_4_results(nodes: List[Any], timeout: float = 3600, poll: float = 0.1) -> None:
    """Block until every node finished learning (``state.round is None``)."""
    deadline = time.monotonic() + timeout
    while not all(n.state.round is None for n in nodes):
        if time.monotonic() > deadline:
            raise TimeoutError("nodes did not finish")
        time.sleep(poll)


def check_equal_models(nodes: List[Any], atol: float = 1e-1) -> None:
    """All learners hold the same parameters (``atol`` like the reference)."""
    first = None
    for node in nodes:
        if node.state.learner is None:
            raise AssertionError("learner not set")
        params = node.state.learner.get_parameters()
        from p2pfl_amd.learning.arena import reading

        with reading(params):  # after the learner's last write on its own stream
            host = {k: v.detach().float().cpu().numpy().copy() for k, v in params.items()}
        if first is None:
            first = host
            continue
        for layer, ref in first.items():
            cur = host[layer]
            if not np.allclose(ref, cur, atol=atol):
                diff = float(np.abs(ref - cur).max())
                raise AssertionError(f"{layer}: {nodes[0].addr} vs {node.addr} differ (max |diff| {diff:.3g})")


def to_numpy(t: torch.Tensor) -> np.ndarray:
    return t.detach().float().cpu().numpy()
