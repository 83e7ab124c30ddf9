"""Message-handler contract (reference ``commands/command.py:24-43``)."""

from __future__ import annotations

import abc


class Command(abc.ABC):
    """A named handler executed by a transport's server side.

    ``execute(source, round, *args)`` for control messages,
    ``execute(source, round, weights=..., contributors=..., weight=...)`` for
    weight messages.  The name returned by :meth:`get_name` is wire-visible.
    """

    @staticmethod
    def get_name() -> str:
        raise NotImplementedError

    @abc.abstractmethod
    def execute(self, source: str, round: int, *args, **kwargs) -> None:
        raise NotImplementedError
