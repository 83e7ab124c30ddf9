"""Per-node mutable learning state (reference ``p2pfl/node_state.py:26-115``).

Field names match the reference (``status``, ``actual_exp_name``, ``round``,
``total_rounds``, ``simulation``, ``learner``, ``models_aggregated``,
``nei_status``, ``train_set``, ``train_set_votes``).  The reference signals
between threads with ``threading.Lock`` objects used as binary semaphores that
other threads release; here each wait has a proper primitive:

* ``model_initialized`` -- ``Event`` set once the initial weights are loaded;
* ``votes_cv``          -- ``Condition`` notified when a vote arrives;
* ``changed``           -- :class:`ChangeSignal`, bumped by every command that
  mutates gossip-relevant state (``models_aggregated``, ``nei_status``) so the
  model gossip loops wake up immediately instead of sleeping a period.
"""

from __future__ import annotations

import threading
from typing import Any, Dict, List, Optional

from p2pfl_amd.utils.lockcheck import make_condition, make_lock


class ChangeSignal:
    """Monotonic version counter with a condition variable."""

    def __init__(self) -> None:
        self._cv = make_condition("ChangeSignal._cv")
        self._version = 0

    @property
    def version(self) -> int:
        return self._version

    def bump(self) -> None:
        with self._cv:
            self._version += 1
            self._cv.notify_all()

    def wait(self, since: int, timeout: float) -> int:
        """Block until the version differs from ``since`` or ``timeout`` elapses."""
        with self._cv:
            if self._version == since and timeout > 0:
                self._cv.wait_for(lambda: self._version != since, timeout=timeout)
            return self._version


class NodeState:
    def __init__(self, addr: str) -> None:
        self.addr = addr
        self.status = "Idle"
        self.actual_exp_name: Optional[str] = None
        self.round: Optional[int] = None
        self.total_rounds: Optional[int] = None
        self.simulation = False

        self.learner: Optional[Any] = None

        self.models_aggregated: Dict[str, List[str]] = {}
        self.nei_status: Dict[str, int] = {}

        self.train_set: List[str] = []
        self.train_set_votes: Dict[str, Dict[str, int]] = {}

        self.train_set_votes_lock = make_lock("NodeState.train_set_votes_lock")
        self.start_thread_lock = make_lock("NodeState.start_thread_lock")
        self.votes_cv = make_condition("NodeState.votes_cv")
        self.model_initialized = threading.Event()
        self.changed = ChangeSignal()

    # -- experiment lifecycle -------------------------------------------
    def set_experiment(self, exp_name: str, total_rounds: int) -> None:
        self.status = "Learning"
        self.actual_exp_name = exp_name
        self.total_rounds = total_rounds
        self.round = 0

    def increase_round(self) -> None:
        if self.round is None:
            raise ValueError("Round not initialized")
        self.round += 1
        self.models_aggregated = {}
        self.changed.bump()

    def clear(self) -> None:
        self.status = "Idle"
        self.actual_exp_name = None
        self.round = None
        self.total_rounds = None
        self.wake_all()

    # -- signalling -----------------------------------------------------
    def notify_vote(self) -> None:
        with self.votes_cv:
            self.votes_cv.notify_all()

    def wake_all(self) -> None:
        """Wake every waiter (used on stop so blocked stages re-check ``round``)."""
        self.notify_vote()
        self.changed.bump()
