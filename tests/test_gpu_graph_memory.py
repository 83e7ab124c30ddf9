"""Step graphs vs the caching allocator (verdict r2 #4, profiles/r3_nan_root_cause.md).

The round-2 NaN of the 8-peer ResNet-50 scenario under rocprofv3 came from
MIOpen's 1x1-convolution path replayed inside a captured step graph: once the
allocator had to map new segments (a profiler allocates), the first replay of
the next fit wrote non-finite weights.  1x1 convolutions now run on the hand-written
implicit-GEMM conv kernels (default) or as native GEMMs over channels-last pixels
(:func:`p2pfl_amd.ops.conv.conv1x1_gemm`, ``P2PFL_CONV1X1_MODE=gemm``).
"""

from __future__ import annotations

import pytest
import torch
import torch.nn.functional as F
from torch import nn

from p2pfl_amd import ops
from p2pfl_amd.ops import conv as conv_ops

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("stride", [1, 2])
def test_conv1x1_gemm_matches_fp32_conv(stride):
    """Forward, input and weight gradients of the 1x1-as-GEMM path vs fp32 F.conv2d on the same bf16 operands."""
    ops.ext()
    g = torch.Generator(device="cuda").manual_seed(7 + stride)
    m = nn.Conv2d(256, 128, 1, stride=stride, bias=False).cuda()
    with torch.no_grad():
        m.weight.copy_(torch.randn(m.weight.shape, device="cuda", generator=g) / 16)
    m = m.to(torch.bfloat16).to(memory_format=torch.channels_last)
    x = torch.randn(4, 256, 14, 14, device="cuda", generator=g).to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last).requires_grad_()
    before = conv_ops.STATS["gemm_1x1_fwd"]
    y = conv_ops.conv1x1_gemm(x, m)
    assert conv_ops.STATS["gemm_1x1_fwd"] == before + 1
    assert y.is_contiguous(memory_format=torch.channels_last)
    dy = torch.randn(y.shape, device="cuda", generator=g).to(torch.bfloat16)
    y.backward(dy)
    xr = x.detach().float().requires_grad_()
    wr = m.weight.detach().float().requires_grad_()
    yr = F.conv2d(xr, wr, None, stride)
    yr.backward(dy.float())
    torch.testing.assert_close(y.float(), yr, atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(m.weight.grad.float(), wr.grad, atol=5e-2, rtol=2e-2)


def test_resnet50_step_graph_survives_poisoned_allocator():
    """Fit (captures the step graph), take every free cached block away and fill it
    with NaN, fit again: the replayed steps must not depend on any of that memory."""
    from p2pfl_amd.data import Cifar10FederatedDM
    from p2pfl_amd.learning.torch_learner import TorchLearner
    from p2pfl_amd.models.resnet import ResNet50
    from p2pfl_amd.utils.alloc_probe import poison_free_blocks

    ops.ext()
    dev = torch.device("cuda", 0)
    ln = TorchLearner(ResNet50(seed=1234), Cifar10FederatedDM(sub_id=0, number_sub=64, partitioner="dirichlet", alpha=0.5),
                      "graph-memory", 1, device=dev)
    ln.fit()
    torch.cuda.synchronize(dev)
    assert ln._step_graph is not None and ln._step_graph.graph is not None, "the fit must replay a captured step graph"
    graph = ln._step_graph.graph
    held = poison_free_blocks(dev, fill=True)
    assert held, "nothing to poison: the allocator had no free cached blocks"
    ln.fit()
    torch.cuda.synchronize(dev)
    assert ln._step_graph.graph is graph  # replayed, not re-captured
    assert bool(torch.isfinite(ln.get_parameters().flat).all())
    del held, ln, graph
    import gc

    gc.collect()  # the learner's graphs go now, not in a later test's capture
    torch.cuda.empty_cache()
