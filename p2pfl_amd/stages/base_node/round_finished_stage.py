"""RoundFinishedStage (reference ``stages/base_node/round_finished_stage.py:34-97``)."""

from __future__ import annotations

from typing import Any, Optional, Type

from p2pfl_amd.management.logger import logger
from p2pfl_amd.settings import Settings
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
        _auto_checkpoint(state)
        state.increase_round()
        logger.round_finished(state.addr)
        for hook in kwargs.get("round_hooks") or ():
            hook(state)
        logger.info(state.addr, f"Round {state.round} of {state.total_rounds} finished.")
        if state.round is None or state.total_rounds is None:
            raise Exception("Round or total rounds not set.")
        if state.round < state.total_rounds:
            return StageFactory.get_stage("TrainStage")
        # last round: a background diffusion (Settings.ASYNC_DIFFUSION) must
        # reach the lagging neighbours before the experiment state is reset
        for diffusion in getattr(state, "diffusions", []):
            diffusion.join()
        state.diffusions = []
        evaluate_and_share(state, communication_protocol)
        # the final metrics must be logged before the experiment counts as finished
        if state.learner is not None:
            state.learner.drain()
        # experiment over: reset per-experiment peer bookkeeping so a new
        # experiment re-gossips the initial model (the reference kept stale
        # nei_status entries and could stall a second experiment)
        state.nei_status = {}
        state.train_set = []
        state.model_initialized.clear()
        state.clear()
        getattr(communication_protocol, "experiment_boundary", lambda: None)()
        logger.info(state.addr, "Training finished!!.")
        return None


def _auto_checkpoint(state: Any) -> None:
    """``Settings.CHECKPOINT_DIR``: persist the round's aggregated model (new; the reference has none)."""
    if not Settings.CHECKPOINT_DIR or state.learner is None:
        return
    import os
    import re

    from p2pfl_amd.learning.checkpoint import save_checkpoint

    safe = re.sub(r"[^A-Za-z0-9_.-]+", "_", str(state.addr))
    path = os.path.join(Settings.CHECKPOINT_DIR, safe, f"round_{state.round}.safetensors")
    meta = {"addr": state.addr, "experiment": state.actual_exp_name, "round": state.round, "total_rounds": state.total_rounds}
    try:
        save_checkpoint(path, state.learner.get_parameters(), meta)
    except Exception as e:  # a full disk must not kill the round
        logger.error(state.addr, f"checkpoint {path} failed: {e}")
