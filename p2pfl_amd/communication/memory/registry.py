"""Process-wide registry of in-memory servers (reference ``memory/server_singleton.py:22-43``).

Unlike the reference singleton, stopping one server removes only that server
(reference quirk Q8: ``InMemoryServer.stop`` reset the whole registry and so
unregistered every other in-process node).
"""

from __future__ import annotations

import itertools
import threading
from typing import Any, Dict, Optional


class InMemoryRegistry:
    _lock = threading.Lock()
    _servers: Dict[str, Any] = {}
    _ids = itertools.count()

    @classmethod
    def register(cls, addr: str, server: Any) -> None:
        with cls._lock:
            if addr in cls._servers and cls._servers[addr] is not server:
                raise Exception(f"Address {addr} already in use")
            cls._servers[addr] = server

    @classmethod
    def unregister(cls, addr: str, server: Any) -> None:
        with cls._lock:
            if cls._servers.get(addr) is server:
                del cls._servers[addr]

    @classmethod
    def get(cls, addr: str) -> Optional[Any]:
        with cls._lock:
            return cls._servers.get(addr)

    @classmethod
    def fresh_address(cls) -> str:
        return f"mem://node-{next(cls._ids)}"

    @classmethod
    def reset(cls) -> None:
        with cls._lock:
            cls._servers.clear()
