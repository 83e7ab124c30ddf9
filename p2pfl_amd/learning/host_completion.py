"""Deferred host work of enqueued GPU passes (asynchronous learners).

The reference's Lightning learner returns from ``fit``/``test`` only after the
work ran, and it reads every metric back on the spot
(``lightning_learner.py:180-230``).  A GPU learner that does the same parks
the node's learning thread on the device's queue for every pass -- and the
stages that follow (adding the model to the aggregator, proposing the pushes
to the train set, waiting for the peers) cannot start until the last kernel
of the epoch finished.

Here a pass is *enqueued*: its loss / accuracy sums are copied into pinned
host memory behind it on the same stream, an event is recorded, and the
metric logging (and, for evaluation, the ``metrics`` broadcast) runs on a
small completion thread once the event fires.  The learning thread moves on
immediately; every consumer of the weights is ordered behind the producing
kernels by the stream, not by the host.  :meth:`HostCompletions.drain` waits
for everything outstanding (end of an experiment, tests).
"""

from __future__ import annotations

import queue
import threading
from typing import Any, Callable, Optional

from p2pfl_amd.management.logger import logger
from p2pfl_amd.utils.lockcheck import make_condition


class HostCompletions:
    """A FIFO of (event, callback): each callback runs after its event completed."""

    def __init__(self, name: str) -> None:
        self.name = name
        self._q: "queue.Queue[Optional[tuple]]" = queue.Queue()
        self._cv = make_condition("HostCompletions._cv")
        self._pending = 0
        self._thread: Optional[threading.Thread] = None

    def submit(self, event: Any, fn: Callable[[], None]) -> None:
        with self._cv:
            self._pending += 1
            if self._thread is None or not self._thread.is_alive():
                self._thread = threading.Thread(target=self._run, name=f"host-completions-{self.name}", daemon=True)
                self._thread.start()
        self._q.put((event, fn))

    def _run(self) -> None:
        while True:
            item = self._q.get()
            if item is None:
                return
            event, fn = item
            try:
                if event is not None:
                    event.synchronize()  # releases the GIL while it waits
                fn()
            except Exception as e:  # a logging failure must not kill the thread
                logger.error(self.name, f"deferred host work failed: {e}")
            finally:
                with self._cv:
                    self._pending -= 1
                    self._cv.notify_all()

    @property
    def pending(self) -> int:
        with self._cv:
            return self._pending

    def drain(self, timeout: Optional[float] = None) -> bool:
        """Wait until every submitted callback ran; False on timeout."""
        with self._cv:
            return self._cv.wait_for(lambda: self._pending == 0, timeout)

    def close(self) -> None:
        self._q.put(None)
