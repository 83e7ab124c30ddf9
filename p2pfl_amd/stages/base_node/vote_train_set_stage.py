"""VoteTrainSetStage (reference ``stages/base_node/vote_train_set_stage.py:36-178``).

Each node casts up to ``TRAIN_SET_SIZE`` weighted random votes, broadcasts
them, waits (condition variable, ``VOTE_TIMEOUT``) for the votes of every
known node, tallies, and takes the top ``TRAIN_SET_SIZE`` with a deterministic
tie-break (name descending, then a stable sort by votes descending: quirk Q11),
so every node computes the same train set.
"""

from __future__ import annotations

import math
import random
import time
from typing import Any, Dict, List, Optional, Type

from p2pfl_amd.commands.vote_train_set_command import VoteTrainSetCommand
from p2pfl_amd.management.logger import logger
from p2pfl_amd.settings import Settings
from p2pfl_amd.stages.stage import Stage
from p2pfl_amd.stages.stage_factory import StageFactory


def tally(votes: Dict[str, Dict[str, int]], k: int) -> List[str]:
    results: Dict[str, int] = {}
    for ballot in votes.values():
        for node, w in ballot.items():
            results[node] = results.get(node, 0) + w
    ordered = sorted(results.items(), key=lambda x: x[0], reverse=True)
    ordered = sorted(ordered, key=lambda x: x[1], reverse=True)
    return [n for n, _ in ordered[: min(len(ordered), k)]]


class VoteTrainSetStage(Stage):
    @staticmethod
    def name() -> str:
        return "VoteTrainSetStage"

    @staticmethod
    def execute(state: Any = None, communication_protocol: Any = None, **kwargs) -> Optional[Type[Stage]]:
        if state is None or communication_protocol is None:
            raise Exception("Invalid parameters on VoteTrainSetStage.")
        VoteTrainSetStage._vote(state, communication_protocol)
        train_set = VoteTrainSetStage._aggregate_votes(state, communication_protocol)
        state.train_set = VoteTrainSetStage._validate_train_set(train_set, state, communication_protocol)
        logger.info(state.addr, f"Train set of {len(state.train_set)} nodes: {state.train_set}")
        if state.addr in state.train_set:
            return StageFactory.get_stage("TrainStage")
        return StageFactory.get_stage("WaitAggregatedModelsStage")

    @staticmethod
    def _vote(state: Any, protocol: Any) -> None:
        candidates = list(protocol.get_neighbors(only_direct=False))
        if state.addr not in candidates:
            candidates.append(state.addr)
        samples = min(Settings.TRAIN_SET_SIZE, len(candidates))
        chosen = random.sample(candidates, samples)
        weights = [math.floor(random.randint(0, 1000) / (i + 1)) for i in range(samples)]
        votes = list(zip(chosen, weights))
        with state.train_set_votes_lock:
            state.train_set_votes[state.addr] = dict(votes)
        logger.debug(state.addr, f"Self Vote: {votes}")
        protocol.broadcast(
            protocol.build_msg(VoteTrainSetCommand.get_name(), [str(x) for v in votes for x in v], round=state.round)
        )

    @staticmethod
    def _aggregate_votes(state: Any, protocol: Any) -> List[str]:
        deadline = time.monotonic() + Settings.VOTE_TIMEOUT
        # check-and-wait under the condition: a vote stored after the check
        # cannot be missed (the handler notifies while holding it)
        with state.votes_cv:
            while True:
                if state.round is None:
                    logger.info(state.addr, "Stopping vote aggregation (learning stopped).")
                    return []
                known = set(protocol.get_neighbors(only_direct=False)) | {state.addr}
                with state.train_set_votes_lock:
                    votes = {k: v for k, v in state.train_set_votes.items() if k in known}
                ready = known == set(votes)
                if ready or time.monotonic() >= deadline:
                    if not ready:
                        logger.info(state.addr, f"Timeout for vote aggregation. Missing votes from {known - set(votes)}")
                    with state.train_set_votes_lock:
                        state.train_set_votes = {}
                    logger.info(state.addr, f"Computed {len(votes)} votes.")
                    return tally(votes, Settings.TRAIN_SET_SIZE)
                state.votes_cv.wait(timeout=min(2.0, max(0.0, deadline - time.monotonic())))

    @staticmethod
    def _validate_train_set(train_set: List[str], state: Any, protocol: Any) -> List[str]:
        live = set(protocol.get_neighbors(only_direct=False)) | {state.addr}
        return [n for n in train_set if n in live]
