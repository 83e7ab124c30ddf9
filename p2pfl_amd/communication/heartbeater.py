"""Heartbeats and failure detection (reference ``communication/heartbeater.py:33-111``).

Every ``HEARTBEAT_PERIOD`` the node broadcasts ``beat <time>`` to its direct
neighbours (flooded onwards by the relay); from the second tick on it evicts
neighbours silent for more than ``HEARTBEAT_TIMEOUT``.  Incoming beats refresh
or add (non-direct discovery) the sender.
"""

from __future__ import annotations

import threading
import time
from typing import Any, Optional

from p2pfl_amd.management.logger import logger
from p2pfl_amd.settings import Settings

heartbeater_cmd_name = "beat"


class Heartbeater(threading.Thread):
    def __init__(self, self_addr: str, neighbors: Any, client: Any) -> None:
        super().__init__(name=f"heartbeater-thread-{self_addr}", daemon=True)
        self._self_addr = self_addr
        self._neighbors = neighbors
        self._client = client
        self._terminate = threading.Event()

    def stop(self) -> None:
        self._terminate.set()

    def beat(self, nei: str, time: float) -> None:
        if nei == self._self_addr:
            return
        self._neighbors.refresh_or_add(nei, time)

    def run(self, period: Optional[float] = None, timeout: Optional[float] = None) -> None:
        check = False
        while not self._terminate.is_set():
            period_ = Settings.HEARTBEAT_PERIOD if period is None else period
            timeout_ = Settings.HEARTBEAT_TIMEOUT if timeout is None else timeout
            t0 = time.time()
            if check:
                for nei, entry in self._neighbors.get_all().items():
                    if t0 - entry.last_beat > timeout_:
                        logger.info(self._self_addr, f"Heartbeat timeout for {nei} ({t0 - entry.last_beat:.2f}s). Removing...")
                        self._neighbors.remove(nei)
            check = True  # first tick only beats; every later tick also checks
            self._client.broadcast(self._client.build_message(heartbeater_cmd_name, args=[str(time.time())]))
            self._terminate.wait(max(0.0, period_ - (time.time() - t0)))
