"""Lock-order checker for the host control plane (lockdep-style race detection).

The reference has no race detection at all (SURVEY §5 "Race detection /
sanitizers"): its threads signal each other with ``threading.Lock`` objects
used as binary semaphores released from other threads (``node_state.py:77-81``,
``aggregator.py:80``/``:145``), and nothing checks that the many locks taken by
command handlers, gossip loops, heartbeaters and learning threads are always
acquired in a consistent order.

Every control-plane lock in this package is created through
:func:`make_lock` / :func:`make_rlock` / :func:`make_condition` with a *class
name* (``"Aggregator._lock"``, ``"Neighbors.neis_lock"``, ...).  With checking
off (the default) these return the plain ``threading`` primitives -- zero
overhead.  With ``P2PFL_LOCKCHECK=1`` in the environment (or :func:`enable`
before nodes are built) they return tracked wrappers that record, per thread,
the stack of held locks and build two acquisition-order graphs:

* a **class graph** (``A -> B`` when a lock of class B is taken while one of
  class A is held).  A cycle through two different classes is a potential
  AB/BA deadlock between *any* instances, even if this run never interleaved
  badly -- the same idea as the Linux kernel's lockdep.
* an **instance graph** for locks of the same class (node 1's aggregator lock
  held while taking node 2's): a cycle there is a potential deadlock between
  in-process peers.

Each new edge keeps the first witness (thread name and a short call-site
stack) so a reported cycle says where both orders were taken.  Long holds
(``hold_warn_s``) are recorded too: a lock held across a blocking send or a
GPU synchronisation stalls every thread that needs it.

``tests/conftest.py`` enables the checker for the whole CPU suite and fails any
test during which a new violation was recorded.
"""

from __future__ import annotations

import os
import threading
import time
import traceback
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Set, Tuple

_raw = threading.Lock  # never tracked: guards the checker's own state


@dataclass
class Violation:
    kind: str  # "class-cycle" | "instance-cycle" | "long-hold"
    cycle: List[str]
    thread: str
    where: str
    witnesses: Dict[str, str] = field(default_factory=dict)

    def __str__(self) -> str:
        s = f"[lockcheck] {self.kind}: {' -> '.join(self.cycle)} (thread {self.thread})\n  at: {self.where}"
        for edge, w in self.witnesses.items():
            s += f"\n  first {edge}: {w}"
        return s


class _Checker:
    def __init__(self) -> None:
        self.enabled = False
        self.raise_on_violation = False
        self.hold_warn_s = 5.0
        self._mu = _raw()
        self._tls = threading.local()
        self.class_edges: Dict[Tuple[str, str], str] = {}
        self.inst_edges: Dict[Tuple[int, int], str] = {}
        self.inst_names: Dict[int, str] = {}
        self.violations: List[Violation] = []
        self._seen_cycles: Set[Tuple[str, ...]] = set()
        self.acquisitions = 0
        self.max_hold: Dict[str, Tuple[float, str]] = {}  # class -> (longest hold s, thread)

    # -- held-lock stack -------------------------------------------------
    def held(self) -> List["_Tracked"]:
        h = getattr(self._tls, "held", None)
        if h is None:
            h = self._tls.held = []
        return h

    @staticmethod
    def _site(skip: int = 3) -> str:
        frames = traceback.extract_stack()[: -skip]
        frames = [f for f in frames if "lockcheck.py" not in f.filename and "threading.py" not in f.filename][-3:]
        return " <- ".join(f"{os.path.basename(f.filename)}:{f.lineno}({f.name})" for f in reversed(frames))

    @staticmethod
    def _path(edges: Set[Tuple[Any, Any]], src: Any, dst: Any) -> Optional[List[Any]]:
        """DFS path src -> dst over ``edges`` (small graphs: tens of nodes)."""
        adj: Dict[Any, List[Any]] = {}
        for a, b in edges:
            adj.setdefault(a, []).append(b)
        stack, prev = [src], {src: None}
        while stack:
            u = stack.pop()
            if u == dst:
                out = [u]
                while prev[out[-1]] is not None:
                    out.append(prev[out[-1]])
                return out[::-1]
            for v in adj.get(u, ()):
                if v not in prev:
                    prev[v] = u
                    stack.append(v)
        return None

    def before_acquire(self, lk: "_Tracked") -> None:
        held = self.held()
        if not held:
            return
        site = None
        with self._mu:
            self.acquisitions += 1
            for h in held:
                if h is lk:
                    continue  # re-entrant RLock / Condition re-acquire
                if h.cls != lk.cls:
                    e = (h.cls, lk.cls)
                    if e not in self.class_edges:
                        site = site or self._site()
                        path = self._path(set(self.class_edges), lk.cls, h.cls)
                        self.class_edges[e] = f"{threading.current_thread().name}: {site}"
                        if path is not None:
                            self._report("class-cycle", path + [lk.cls], site, self.class_edges, path)
                else:
                    e2 = (id(h), id(lk))
                    self.inst_names[id(h)] = f"{h.cls}#{id(h) & 0xFFFF:04x}"
                    self.inst_names[id(lk)] = f"{lk.cls}#{id(lk) & 0xFFFF:04x}"
                    if e2 not in self.inst_edges:
                        site = site or self._site()
                        path = self._path(set(self.inst_edges), id(lk), id(h))
                        self.inst_edges[e2] = f"{threading.current_thread().name}: {site}"
                        if path is not None:
                            names = [self.inst_names.get(p, str(p)) for p in path + [id(lk)]]
                            self._report("instance-cycle", names, site, self.inst_edges, path)

    def _report(self, kind: str, cycle: List[Any], site: str, edges: Dict[Any, str], path: List[Any]) -> None:
        key = (kind,) + tuple(sorted(map(str, cycle)))
        if key in self._seen_cycles:
            return
        self._seen_cycles.add(key)
        wit = {}
        for a, b in zip(path, path[1:]):
            na = self.inst_names.get(a, a) if kind == "instance-cycle" else a
            nb = self.inst_names.get(b, b) if kind == "instance-cycle" else b
            wit[f"{na} -> {nb}"] = edges.get((a, b), "?")
        v = Violation(kind, [str(c) for c in cycle], threading.current_thread().name, site, wit)
        self.violations.append(v)
        if self.raise_on_violation:
            raise LockOrderError(str(v))

    def after_acquire(self, lk: "_Tracked") -> None:
        lk._t_acq = time.monotonic()
        lk._owner = threading.get_ident()
        held = self.held()
        lk._held_in = held
        held.append(lk)

    def on_release(self, lk: "_Tracked") -> None:
        # The owner's stack, not the caller's: a Lock used as a semaphore may
        # legally be released by another thread (reference node_state.py:81).
        held = getattr(lk, "_held_in", None) or self.held()
        for i in range(len(held) - 1, -1, -1):
            if held[i] is lk:
                del held[i]
                break
        lk._held_in = None
        dt = time.monotonic() - getattr(lk, "_t_acq", time.monotonic())
        prev = self.max_hold.get(lk.cls)
        if prev is None or dt > prev[0]:
            self.max_hold[lk.cls] = (dt, threading.current_thread().name)
        if dt > self.hold_warn_s and lk.cls not in _HOLD_EXEMPT:
            with self._mu:
                self.violations.append(
                    Violation("long-hold", [lk.cls], threading.current_thread().name, f"held {dt:.2f} s; {self._site()}")
                )

    def reset(self) -> None:
        with self._mu:
            self.class_edges.clear()
            self.inst_edges.clear()
            self.inst_names.clear()
            self.violations.clear()
            self._seen_cycles.clear()
            self.acquisitions = 0
            self.max_hold.clear()


class LockOrderError(RuntimeError):
    pass


_checker = _Checker()
_HOLD_EXEMPT: Set[str] = set()


class _Tracked:
    """Common wrapper around a ``_thread`` lock; also usable under ``Condition``."""

    def __init__(self, inner: Any, cls: str) -> None:
        self._inner = inner
        self.cls = cls
        self._owner: Optional[int] = None
        self._held_in: Optional[List["_Tracked"]] = None
        self._t_acq = 0.0

    def acquire(self, blocking: bool = True, timeout: float = -1) -> bool:
        if _checker.enabled and blocking:
            _checker.before_acquire(self)
        ok = self._inner.acquire(blocking, timeout)
        if ok and _checker.enabled:
            _checker.after_acquire(self)
        return ok

    def release(self) -> None:
        if _checker.enabled:
            _checker.on_release(self)
        self._inner.release()

    __enter__ = acquire

    def __exit__(self, *exc: Any) -> None:
        self.release()

    def locked(self) -> bool:
        return self._inner.locked()

    def __repr__(self) -> str:
        return f"<tracked {self.cls} {self._inner!r}>"


class TrackedLock(_Tracked):
    def __init__(self, cls: str) -> None:
        super().__init__(_raw(), cls)

    # Condition(lock) protocol: plain Lock has no recursion state.
    def _release_save(self) -> None:
        self.release()

    def _acquire_restore(self, _state: Any) -> None:
        self.acquire()

    def _is_owned(self) -> bool:
        return self._inner.locked() and self._owner == threading.get_ident()


class TrackedRLock(_Tracked):
    def __init__(self, cls: str) -> None:
        super().__init__(threading.RLock(), cls)
        self._depth = 0

    def acquire(self, blocking: bool = True, timeout: float = -1) -> bool:
        outer = not self._inner._is_owned()
        if _checker.enabled and blocking and outer:
            _checker.before_acquire(self)
        ok = self._inner.acquire(blocking, timeout)
        if ok:
            self._depth += 1
            if outer and _checker.enabled:
                _checker.after_acquire(self)
        return ok

    __enter__ = acquire

    def release(self) -> None:
        self._depth -= 1
        if self._depth == 0 and _checker.enabled:
            _checker.on_release(self)
        self._inner.release()

    def locked(self) -> bool:
        return self._depth > 0

    def _release_save(self) -> Any:
        depth, self._depth = self._depth, 0
        if _checker.enabled:
            _checker.on_release(self)
        return depth, self._inner._release_save()

    def _acquire_restore(self, state: Any) -> None:
        depth, inner_state = state
        if _checker.enabled:
            _checker.before_acquire(self)
        self._inner._acquire_restore(inner_state)
        self._depth = depth
        if _checker.enabled:
            _checker.after_acquire(self)

    def _is_owned(self) -> bool:
        return self._inner._is_owned()


# -- public factories ---------------------------------------------------------
def make_lock(name: str) -> Any:
    return TrackedLock(name) if _checker.enabled else threading.Lock()


def make_rlock(name: str) -> Any:
    return TrackedRLock(name) if _checker.enabled else threading.RLock()


def make_condition(name: str, lock: Any = None) -> threading.Condition:
    if lock is None:
        lock = make_rlock(name)
    return threading.Condition(lock)


def enable(raise_on_violation: bool = False, hold_warn_s: float = 5.0, exempt: Optional[Set[str]] = None) -> None:
    """Track every lock created from now on (existing plain locks stay untracked)."""
    _checker.enabled = True
    _checker.raise_on_violation = raise_on_violation
    _checker.hold_warn_s = hold_warn_s
    if exempt:
        _HOLD_EXEMPT.update(exempt)


def disable() -> None:
    _checker.enabled = False


def is_enabled() -> bool:
    return _checker.enabled


def reset() -> None:
    _checker.reset()


def violations() -> List[Violation]:
    with _checker._mu:
        return list(_checker.violations)


def max_holds() -> Dict[str, Tuple[float, str]]:
    """Longest observed hold per lock class: ``{class: (seconds, thread name)}``."""
    with _checker._mu:
        return dict(_checker.max_hold)


def report() -> Dict[str, Any]:
    """Observed order graph and violations (for logs / CI artefacts)."""
    with _checker._mu:
        return {
            "enabled": _checker.enabled,
            "acquisitions_while_holding": _checker.acquisitions,
            "class_edges": sorted(f"{a} -> {b}" for a, b in _checker.class_edges),
            "max_hold_s": {k: round(v[0], 4) for k, v in sorted(_checker.max_hold.items())},
            "violations": [str(v) for v in _checker.violations],
        }


if os.environ.get("P2PFL_LOCKCHECK", "") not in ("", "0"):
    enable(raise_on_violation=os.environ.get("P2PFL_LOCKCHECK") == "raise")
