"""Stage runner (reference ``stages/workflows.py:28-55``).

Runs ``stage.execute(**kwargs)`` until a stage returns ``None``.  Each stage
execution is recorded as a tracer span (``stage:<Name>``) so per-round
wall-clock can be broken down by stage.
"""

from __future__ import annotations

from typing import Optional, Type

from p2pfl_amd.management.logger import logger
from p2pfl_amd.stages.stage import Stage
from p2pfl_amd.stages.stage_factory import StageFactory


class StageWorkflow:
    def __init__(self, first_stage: Type[Stage]) -> None:
        self.first_stage = first_stage
        self.current_stage = first_stage

    def run(self, **kwargs) -> None:
        state = kwargs.get("state")
        if state is None:
            raise ValueError("State not found in kwargs")
        self.current_stage = self.first_stage
        while True:
            name = self.current_stage.name()
            logger.debug(state.addr, f"Running stage: {name}")
            with logger.span(state.addr, f"stage:{name}", round=state.round):
                nxt: Optional[Type[Stage]] = self.current_stage.execute(**kwargs)
            if nxt is None:
                break
            self.current_stage = nxt


StageWokflow = StageWorkflow  # reference spelling


class LearningWorkflow(StageWorkflow):
    def __init__(self) -> None:
        super().__init__(StageFactory.get_stage("StartLearningStage"))
