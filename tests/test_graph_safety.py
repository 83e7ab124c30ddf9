"""CPU checks of the round-3 graph-safety and split-K helpers (no GPU needed)."""

from __future__ import annotations

import gc

import torch
from torch import nn

from p2pfl_amd.learning.step_graph import no_gc
from p2pfl_amd.ops import conv as conv_ops
from p2pfl_amd.ops.splitk import slab_elems, tiles_of


def test_no_gc_disables_collection_during_capture_and_restores():
    assert gc.isenabled()
    with no_gc():
        assert not gc.isenabled()
    assert gc.isenabled()
    gc.disable()
    try:
        with no_gc():
            assert not gc.isenabled()
        assert not gc.isenabled()  # a caller that had GC off keeps it off
    finally:
        gc.enable()


def test_slab_elems_covers_fragment_native_tiles():
    # one 128 x 128 tile per started tile row / column (tails included)
    assert slab_elems(128, 128) == 128 * 128
    assert slab_elems(130, 64) == tiles_of(130, 64) * 128 * 128 == 2 * 128 * 128
    assert slab_elems(6304, 768) == 50 * 6 * 128 * 128
    # the 256 x 256 variant (bit 6) and the ping-pong kernel's row-major slabs
    assert slab_elems(300, 300, 64) == 2 * 2 * 256 * 256
    assert slab_elems(768, 768, 2048) >= 768 * 768


def test_conv1x1_gemm_matches_conv2d_on_cpu():
    """1x1 convolutions as GEMMs over channels-last pixels (stride 1 and 2), values and gradients."""
    torch.manual_seed(0)
    for s in (1, 2):
        m = nn.Conv2d(16, 24, 1, stride=s, bias=False)
        x = torch.randn(2, 16, 9, 9).contiguous(memory_format=torch.channels_last).requires_grad_()
        y = conv_ops.conv1x1_gemm(x, m)
        xr = x.detach().clone().requires_grad_()
        yr = m(xr)
        torch.testing.assert_close(y, yr)
        g = torch.randn_like(yr)
        y.backward(g)
        wg = m.weight.grad.clone()
        m.weight.grad = None
        yr.backward(g)
        torch.testing.assert_close(x.grad, xr.grad)
        torch.testing.assert_close(wg, m.weight.grad)
        assert y.is_contiguous(memory_format=torch.channels_last)


def test_1x1_routing_is_gpu_only():
    m = nn.Conv2d(16, 24, 1, bias=False)
    assert not conv_ops._is_1x1(torch.randn(1, 16, 4, 4), m)  # CPU tensors keep nn.Conv2d
