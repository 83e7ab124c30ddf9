"""Kernel-choice policy (p2pfl_amd/ops/autotune.py) and split-K helpers, CPU side."""

from __future__ import annotations

import pytest

from p2pfl_amd.ops import autotune
from p2pfl_amd.ops.splitk import IN_LAUNCH_MAX_SPLITS, tiles_of


@pytest.mark.parametrize("val,expect", [("1", "native"), ("native", "native"), ("0", "library"), ("off", "library"),
                                        ("auto", "auto"), ("", "auto"), ("bogus", "auto")])
def test_policy_parsing(monkeypatch, val, expect):
    monkeypatch.setenv("P2PFL_TEST_POLICY", val)
    assert autotune.policy("P2PFL_TEST_POLICY") == expect


def test_policy_default_is_auto(monkeypatch):
    monkeypatch.delenv("P2PFL_TEST_POLICY", raising=False)
    assert autotune.policy("P2PFL_TEST_POLICY") == "auto"


def test_cached_choice_is_reused_without_timing():
    autotune.reset()
    autotune._CHOICE[("k",)] = "library"
    calls = []
    assert autotune.choose(("k",), [("native", lambda: calls.append(1)), ("library", lambda: calls.append(2))]) == "library"
    assert calls == []
    assert "library" in autotune.summary() or autotune.summary() == "('k',): library ()"
    autotune.reset()
    assert autotune.choices() == {}


def test_split_k_helpers():
    assert tiles_of(128, 128) == 1 and tiles_of(129, 128) == 2 and tiles_of(6304, 768) == 50 * 6
    assert 1 < IN_LAUNCH_MAX_SPLITS <= 8


def test_conv_split_choices():
    from p2pfl_amd.ops.conv import mn_splits, out_hw, wgrad_splits

    assert out_hw(32, 32, (3, 3), 1, 1, 1) == (32, 32)
    assert out_hw(32, 32, (3, 3), 2, 1, 1) == (16, 16)
    assert out_hw(9, 9, (1, 1), 2, 0, 1) == (5, 5)
    # big output grids need no split, small ones are split until ~1 WG per CU
    assert mn_splits(32768, 64, 576) == 1
    assert mn_splits(512, 512, 4608) == 16
    assert wgrad_splits(64, 576, 32768) >= 16


def test_conv_tuning_candidates(monkeypatch):
    """The per-shape conv candidates: every tuned variant x split option; untuned only the
    default variant; the stride-2 by-phase path offered for k > 1 only."""
    from p2pfl_amd.ops import conv as cv

    make = lambda v, sp: (v, sp)  # noqa: E731
    monkeypatch.setattr(cv, "_TUNE", True)
    c = cv._configs("gather", make, 10, (1, 2))
    assert c == {f"gather_v{v}_s{sp}": (v, sp) for v in cv._TUNE_VARIANTS for sp in (1, 2)}
    monkeypatch.setattr(cv, "_TUNE", False)
    assert cv._configs("", make, 10, (4,)) == {"v10_s4": (10, 4)}
    assert cv._split_options(1, 512) == (1, 2, 4)
    assert cv._split_options(8, 1152) == (8,)
    assert cv.s2_phases_ok(2, 1, [32, 32, 32, 64]) and not cv.s2_phases_ok(2, 1, [32, 32, 32, 64], (1, 1))
    assert not cv.s2_phases_ok(1, 1, [32, 32, 32, 64]) and not cv.s2_phases_ok(2, 1, [2, 9, 9, 64])


def test_split_k_counters_of_a_captured_graph_come_from_its_own_ring():
    """Two graphs captured on one pooled stream must never share counter slices
    (concurrent replays would corrupt each other's tile counts); eager launches
    keep using the per-stream ring."""
    import pytest
    import torch

    from p2pfl_amd.ops import splitk

    dev = torch.device("cpu")
    a, b = splitk.GraphCounters(dev, 64), splitk.GraphCounters(dev, 64)
    with splitk.graph_scope(a):
        s1 = splitk.counters(10, dev)
        s2 = splitk.counters(10, dev)
        with splitk.graph_scope(b):
            s3 = splitk.counters(10, dev)
    assert s1.data_ptr() != s2.data_ptr() and s1.untyped_storage().data_ptr() == a.buf.untyped_storage().data_ptr()
    assert s3.untyped_storage().data_ptr() == b.buf.untyped_storage().data_ptr()
    assert getattr(splitk._SCOPE, "ring", None) is None
    with splitk.graph_scope(a), pytest.raises(RuntimeError, match="exhausted"):
        splitk.counters(60, dev)  # a graph's ring never wraps onto slices it already baked in


def test_gemm_variant_rule_takes_the_ping_pong_kernel_for_large_products():
    import importlib

    gemm = importlib.import_module("p2pfl_amd.ops.gemm")

    assert gemm._variant(True, 1, 6304, 2304, 768) == gemm.PP  # ViT QKV forward: 225 tiles of 256^2
    assert gemm._variant(True, 1, 6304, 768, 768) == 10  # 75 tiles: the 128 x 128 tile
    assert gemm._variant(True, 1, 8192, 8192, 8192, False) == gemm.PP
    assert gemm._variant(True, 1, 8192, 8192, 8008) != gemm.PP  # k-major K tail
    assert gemm._variant(False, 1, 8192, 8192, 6304, False) == gemm.PP  # m/n-major tails are range-checked
    assert gemm._variant(False, 4, 768, 768, 6304, False) == 2  # split-K weight gradient
