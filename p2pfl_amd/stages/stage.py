"""Stage contract (reference ``stages/stage.py:23-34``)."""

from __future__ import annotations

from typing import Optional, Type


class Stage:
    @staticmethod
    def name() -> str:
        raise NotImplementedError("Stage name not implemented.")

    @staticmethod
    def execute(**kwargs) -> Optional[Type["Stage"]]:
        raise NotImplementedError("Stage execute not implemented.")
