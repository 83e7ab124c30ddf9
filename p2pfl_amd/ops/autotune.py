"""Per-shape choice between a hand-written kernel and the ROCm library path.

The hand-written MFMA GEMM / implicit-GEMM convolution (``csrc/gemm_core.h``)
and the library (hipBLASLt / MIOpen) win on different shapes: the native core
is fastest where its fused epilogues or split-K reductions pay, the library's
deeper-pipelined 256-wide tiles where a shape is large and regular.  Instead
of a fixed rule, the first eager call of each shape times both candidates
(after one warm-up each, HIP events, a few repetitions) and the faster one is
used from then on -- including inside the HIP graphs captured later, which
replay whatever the eager step chose.

Policy per op family (environment, read once):
    P2PFL_NATIVE_CONV / P2PFL_NATIVE_GEMM = "1" always native, "0" always
    library, unset or "auto" -> measured choice (the default).
``choices()`` returns the decisions taken so far (logged by the benches).
"""

from __future__ import annotations

import os
import threading
from typing import Callable, Dict, Hashable, Optional, Sequence, Tuple

import torch

_LOCK = threading.Lock()
_CHOICE: Dict[Hashable, str] = {}
_TIMES: Dict[Hashable, Dict[str, float]] = {}
PASSES = max(1, int(os.environ.get("P2PFL_AUTOTUNE_PASSES", "3")))


def policy(env: str) -> str:
    v = os.environ.get(env, "auto").strip().lower()
    if v in ("1", "native", "on"):
        return "native"
    if v in ("0", "library", "off"):
        return "library"
    return "auto"


def _time(fn: Callable[[], object], iters: int) -> float:
    """GPU time per call, not host launch time: the stream is first parked on a
    spin kernel long enough for the host to enqueue every timed call, so the
    calls then run back to back on the device (as they do in a replayed HIP
    graph, where these choices end up)."""
    import time

    fn()  # warm-up (library solver search, lazy workspaces)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    host = time.perf_counter() - t0  # upper bound on one call's enqueue time
    start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(int(max(2e6, 2.6e9 * host * (iters + 2))))  # ~cycles at 2.6 GHz
    start.record()
    for _ in range(iters):
        fn()
    end.record()
    end.synchronize()
    return start.elapsed_time(end) / iters


def choose(key: Hashable, candidates: Sequence[Tuple[str, Callable[[], object]]], iters: int = 5,
           default: Optional[str] = None) -> str:
    """Name of the faster candidate for ``key`` (timed once, then cached).

    During a HIP-graph capture nothing can be timed: an unseen key then takes
    ``default`` (or the first candidate) without caching it.
    """
    got = _CHOICE.get(key)
    if got is not None:
        return got
    if torch.cuda.is_current_stream_capturing():
        return default or candidates[0][0]
    with _LOCK:
        got = _CHOICE.get(key)
        if got is not None:
            return got
        # round-robin passes, best of each candidate: the chip's clock ramps and
        # settles over milliseconds (DVFS), so one pass in a fixed order times the
        # first candidates at a different clock than the last ones
        times: Dict[str, float] = {}
        for k in range(PASSES):
            order = list(candidates[k % len(candidates):]) + list(candidates[: k % len(candidates)])
            for name, fn in order:
                t = _time(fn, iters)
                times[name] = min(times.get(name, t), t)
        best = min(times, key=times.get)
        _CHOICE[key] = best
        _TIMES[key] = times
        return best


def choices() -> Dict[Hashable, Tuple[str, Dict[str, float]]]:
    return {k: (v, dict(_TIMES.get(k, {}))) for k, v in _CHOICE.items()}


def summary() -> str:
    """One line per decided shape: key, choice, timings (ms)."""
    lines = []
    for k, (v, t) in choices().items():
        ts = ", ".join(f"{n} {ms:.3f}" for n, ms in sorted(t.items()))
        lines.append(f"{k}: {v} ({ts})")
    return "\n".join(lines)


def reset() -> None:
    with _LOCK:
        _CHOICE.clear()
        _TIMES.clear()
