"""CPU test of the step-graph capture protocol (no GPU: torch.cuda is faked).

The warm-up step of a capture does the expensive first-use work (autotune
timing, library solver choice) and must run under the SHARED device gate, so
other virtual peers keep training; only the recording holds the gate
exclusively and ``StepGraph._CAPTURE_LOCK``.  A warm-up slower than the lock
checker's long-hold limit must therefore not register a long hold
(an 11 s hold stopped the driver's GPU suite).
"""

from __future__ import annotations

import contextlib
import threading
import time
import types

import pytest
import torch

from p2pfl_amd.learning import step_graph
from p2pfl_amd.utils import lockcheck


class _FakeStream:
    def wait_stream(self, other):
        pass

    def synchronize(self):
        pass


class _FakeMT:
    def __init__(self, params):
        self.params = params

    def fill_grad_table(self, gtab):
        pass


class _FakeOpt:
    def __init__(self, params):
        self.mt = _FakeMT(params)
        self.t = 0
        self.state = torch.zeros(4)

    def config(self):
        return ("fake",)

    def state_tensors(self):
        return [self.state]


@pytest.fixture
def fake_cuda(monkeypatch):
    monkeypatch.setattr(step_graph, "private_stream", lambda *a, **k: _FakeStream())
    monkeypatch.setattr(torch.cuda, "current_stream", lambda *a, **k: _FakeStream())
    monkeypatch.setattr(torch.cuda, "stream", lambda s: contextlib.nullcontext())
    monkeypatch.setattr(torch.cuda, "synchronize", lambda *a, **k: None)
    monkeypatch.setattr(torch.cuda, "CUDAGraph", lambda: types.SimpleNamespace(replay=lambda: None))
    monkeypatch.setattr(torch.cuda, "graph", lambda *a, **k: contextlib.nullcontext())
    monkeypatch.setattr(step_graph.splitk, "GraphCounters", lambda dev: None)
    monkeypatch.setattr(step_graph.splitk, "graph_scope", lambda c: contextlib.nullcontext())


def _make_graph():
    p = torch.nn.Parameter(torch.ones(3))
    arena = types.SimpleNamespace(flat=torch.ones(8), shadow=None, _int_buffers={"nb": torch.zeros(1, dtype=torch.int64)})
    learner = types.SimpleNamespace(device=torch.device("cpu"), arena=arena, model=object())
    loader = types.SimpleNamespace(batch_size=4, x=torch.zeros(16, 2), y=torch.zeros(16, dtype=torch.int64))
    return step_graph.TrainStepGraph(learner, _FakeOpt([p]), loader), arena


def _wkey(sg):
    return ("train", type(sg.learner.model).__name__, sg.B, tuple(sg.loader.x.shape[1:]), sg.opt.config())


def test_first_warmup_of_a_model_runs_alone_later_ones_shared(fake_cuda, monkeypatch):
    """The first warm-up of a model structure takes the gate exclusively (its
    autotune timings see no other peer's kernels); the next peer's
    warm-up of the same structure runs under the shared gate."""
    sg, arena = _make_graph()
    monkeypatch.setattr(step_graph, "_WARMED", set())
    gate = step_graph.GATE
    seen = []

    def body(graph):
        if not graph:
            seen.append((gate._excl, gate._shared))
        return torch.zeros(())

    monkeypatch.setattr(sg, "_body", body)
    sg.capture(torch.arange(4))
    assert seen[0] == (True, 0), seen
    assert _wkey(sg) in step_graph._WARMED
    sg2, _ = _make_graph()
    monkeypatch.setattr(sg2, "_body", body)
    sg2.capture(torch.arange(4))
    assert seen[1][0] is False and seen[1][1] >= 1, seen


def test_slow_warmup_runs_under_shared_gate_and_does_not_hold_capture_lock(fake_cuda, monkeypatch):
    if not lockcheck.is_enabled():
        pytest.skip("P2PFL_LOCKCHECK=0")
    sg, arena = _make_graph()
    # a later peer's warm-up (the model structure was warmed up once already)
    monkeypatch.setattr(step_graph, "_WARMED", {_wkey(sg)})
    seen = {}
    gate = step_graph.GATE

    def body(graph):
        if not graph:
            seen["warm_shared"] = gate._shared
            seen["warm_excl"] = gate._excl
            arena.flat.add_(5.0)  # the warm-up step moves the weights ...
            arena._int_buffers["nb"].add_(1)
            time.sleep(1.5)  # ... and is slow (first-use work)
        else:
            seen["rec_excl"] = gate._excl
        return torch.zeros(())

    monkeypatch.setattr(sg, "_body", body)
    # another peer's step may run while this peer warms up
    other_ran = threading.Event()

    def other_peer():
        time.sleep(0.1)
        with gate.shared():
            other_ran.set()

    t = threading.Thread(target=other_peer)
    old = lockcheck._checker.hold_warn_s
    before = len(lockcheck.violations())
    lockcheck._checker.hold_warn_s = 1.0
    try:
        t.start()
        sg.capture(torch.arange(4))
        t.join(5)
    finally:
        lockcheck._checker.hold_warn_s = old
    assert seen["warm_shared"] >= 1 and not seen["warm_excl"], "warm-up must run under the shared gate"
    assert seen["rec_excl"], "the recording must hold the gate exclusively"
    assert other_ran.is_set() and not t.is_alive(), "another peer's step was blocked by the warm-up"
    holds = [v for v in lockcheck.violations()[before:] if v.kind == "long-hold"]
    assert not holds, holds
    assert lockcheck.max_holds()["StepGraph._CAPTURE_LOCK"][0] < 1.0
    # the warm-up's effects on the weights / integer buffers are undone
    assert torch.equal(arena.flat, torch.ones(8)) and int(arena._int_buffers["nb"]) == 0
    assert sg.graph is not None
