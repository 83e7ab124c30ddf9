"""``beat <time>`` handler (reference ``commands/heartbeat_command.py:27-52``)."""

from __future__ import annotations

from typing import Any, Optional

from p2pfl_amd.commands.command import Command


class HeartbeatCommand(Command):
    def __init__(self, heartbeat: Any) -> None:
        self._heartbeat = heartbeat

    @staticmethod
    def get_name() -> str:
        return "beat"

    def execute(self, source: str, round: int, time: Optional[str] = None, *args, **kwargs) -> None:
        if time is None:
            raise ValueError("Time is required")
        self._heartbeat.beat(source, time=float(time))
