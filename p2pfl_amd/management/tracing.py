"""Lightweight span tracer (new; the reference has no tracing).

Every stage execution, gossip iteration and aggregation is recorded as a span
``(node, name, t_start, duration, attrs)``.  Spans can be summarised per name
or exported as a Chrome/Perfetto trace (``chrome://tracing``) so control-plane
latency can be lined up against ``rocprofv3`` kernel traces of the same run.
Byte counters record how much model data each node pushed/pulled.
"""

from __future__ import annotations

import contextlib
import json
import threading
import time
from collections import defaultdict
from dataclasses import dataclass, field
from typing import Any, Dict, Iterator, List, Optional


@dataclass
class Span:
    node: str
    name: str
    start: float
    duration: float
    thread: str
    attrs: Dict[str, Any] = field(default_factory=dict)


class Tracer:
    """Thread-safe span / counter recorder."""

    def __init__(self, max_spans: int = 200_000) -> None:
        self._lock = threading.Lock()
        self._spans: List[Span] = []
        self._counters: Dict[str, Dict[str, float]] = defaultdict(lambda: defaultdict(float))
        self.max_spans = max_spans
        self.enabled = True

    @contextlib.contextmanager
    def span(self, node: str, name: str, **attrs: Any) -> Iterator[Dict[str, Any]]:
        if not self.enabled:
            yield attrs
            return
        t0 = time.perf_counter()
        try:
            yield attrs
        finally:
            dt = time.perf_counter() - t0
            sp = Span(node, name, t0, dt, threading.current_thread().name, dict(attrs))
            with self._lock:
                if len(self._spans) < self.max_spans:
                    self._spans.append(sp)

    def record(self, node: str, name: str, start: float, duration: float, **attrs: Any) -> None:
        """Add a span measured by the caller (``start`` on the ``perf_counter`` clock)."""
        if not self.enabled:
            return
        sp = Span(node, name, start, duration, threading.current_thread().name, dict(attrs))
        with self._lock:
            if len(self._spans) < self.max_spans:
                self._spans.append(sp)

    def count(self, node: str, key: str, value: float = 1.0) -> None:
        with self._lock:
            self._counters[node][key] += value

    def counters(self, node: Optional[str] = None) -> Dict[str, Any]:
        with self._lock:
            if node is not None:
                return dict(self._counters.get(node, {}))
            return {n: dict(c) for n, c in self._counters.items()}

    def spans(self, node: Optional[str] = None, name: Optional[str] = None) -> List[Span]:
        with self._lock:
            return [s for s in self._spans if (node is None or s.node == node) and (name is None or s.name == name)]

    def summary(self) -> Dict[str, Dict[str, float]]:
        """Per span name: count, total, mean, max (seconds)."""
        out: Dict[str, Dict[str, float]] = {}
        for s in self.spans():
            d = out.setdefault(s.name, {"count": 0, "total_s": 0.0, "max_s": 0.0})
            d["count"] += 1
            d["total_s"] += s.duration
            d["max_s"] = max(d["max_s"], s.duration)
        for d in out.values():
            d["mean_s"] = d["total_s"] / max(1, d["count"])
        return out

    def export_chrome_trace(self, path: str) -> None:
        events = []
        tids: Dict[str, int] = {}
        for s in self.spans():
            tid = tids.setdefault(s.thread, len(tids))
            events.append(
                {
                    "name": s.name,
                    "ph": "X",
                    "ts": s.start * 1e6,
                    "dur": s.duration * 1e6,
                    "pid": s.node,
                    "tid": tid,
                    "args": {k: str(v) for k, v in s.attrs.items()},
                }
            )
        with open(path, "w") as f:
            json.dump({"traceEvents": events}, f)

    def clear(self) -> None:
        with self._lock:
            self._spans.clear()
            self._counters.clear()


tracer = Tracer()
