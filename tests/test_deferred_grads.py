"""ops.fused.deferred_param_grads bookkeeping on the CPU (the GPU reduction itself is
tested against the per-pass reductions in tests/test_gpu_fused_ops.py)."""

from __future__ import annotations

import threading

import torch

from p2pfl_amd.ops import fused


class _FakeFx:
    def __init__(self) -> None:
        self.calls = 0

    def col_reduce_multi(self, parts, outs):
        self.calls += 1
        for p, o in zip(parts, outs):
            o.copy_(p.sum(0).to(o.dtype))

    @staticmethod
    def colsum_splits(n):
        return 2

    def column_sum_parts_multi(self, xs, parts):
        self.calls += 1
        for x, p in zip(xs, parts):
            p.zero_()
            p[0].copy_(x.float().sum(0))


def _patch(monkeypatch) -> _FakeFx:
    fx = _FakeFx()
    monkeypatch.setattr(fused, "_fx", lambda: fx)
    monkeypatch.setattr(fused, "_DEFER_ON", True)
    return fx


def test_flush_assigns_and_accumulates_grads(monkeypatch):
    fx = _patch(monkeypatch)
    w = torch.nn.Parameter(torch.zeros(4))
    b = torch.nn.Parameter(torch.zeros(4, dtype=torch.bfloat16))
    b.grad = torch.ones(4, dtype=torch.bfloat16)  # an existing gradient is accumulated into
    pw, pb = torch.arange(12.0).view(3, 4), torch.ones(2, 4)
    with fused.deferred_param_grads():
        d = fused.defer_scope()
        assert d is not None
        assert fused.defer_grad(d, w, pw) and fused.defer_grad(d, b, pb)
        assert w.grad is None  # nothing before the exit
    assert fx.calls == 1
    torch.testing.assert_close(w.grad, pw.sum(0))
    assert b.grad.dtype == torch.bfloat16 and torch.equal(b.grad.float(), torch.full((4,), 3.0))
    assert fused.defer_scope() is None


def test_scope_is_closed_after_exit_and_refuses_non_parameters(monkeypatch):
    fx = _patch(monkeypatch)
    with fused.deferred_param_grads():
        d = fused.defer_scope()
        assert not fused.defer_grad(d, torch.zeros(4), torch.ones(2, 4))  # not a leaf Parameter
    assert fx.calls == 0  # nothing collected: no launch
    p = torch.nn.Parameter(torch.zeros(4))
    assert not fused.defer_grad(d, p, torch.ones(2, 4))  # a backward after the flush reduces in place
    assert not fused.defer_grad(None, p, torch.ones(2, 4))


def test_scopes_are_per_thread_and_disabled_by_the_switch(monkeypatch):
    _patch(monkeypatch)
    seen = []
    with fused.deferred_param_grads():
        t = threading.Thread(target=lambda: seen.append(fused.defer_scope()))
        t.start()
        t.join()
        assert fused.defer_scope() is not None
    assert seen == [None]  # another peer's thread never records this step's collection
    monkeypatch.setattr(fused, "_DEFER_ON", False)
    with fused.deferred_param_grads():
        assert fused.defer_scope() is None
    with fused.deferred_param_grads(enabled=False):
        assert fused.defer_scope() is None


def test_deferred_column_sums_of_activations(monkeypatch):
    fx = _patch(monkeypatch)
    b = torch.nn.Parameter(torch.zeros(8, dtype=torch.bfloat16))
    x = torch.randn(5, 8).to(torch.bfloat16)
    with fused.deferred_param_grads():
        d = fused.defer_scope()
        assert fused.defer_colsum(d, b, x)
        assert not fused.defer_colsum(d, b, x.t())  # not a contiguous [N, H] activation
    assert fx.calls == 2  # one partial pass + one reduction for all deferred sums
    torch.testing.assert_close(b.grad.float(), x.float().sum(0), atol=0.05, rtol=0.01)
