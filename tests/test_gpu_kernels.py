"""Numerics of the HIP kernels vs plain-PyTorch fp32 references (MI355X only)."""

from __future__ import annotations

import pytest
import torch

from p2pfl_amd import ops

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _require_ext():
    ops.ext()  # fail loudly if the native extension is missing on a GPU box


@pytest.mark.parametrize("k", [1, 2, 3, 8, 16, 21])
@pytest.mark.parametrize("n", [64, 4096 + 4, 6_497_216])
def test_weighted_sum(k, n):
    g = torch.Generator(device="cuda").manual_seed(k * 7 + n % 13)
    flats = [torch.randn(n, device="cuda", generator=g) for _ in range(k)]
    weights = [float(i % 5 + 1) for i in range(k)]
    out = ops.weighted_average(flats, weights)
    ref = ops.weighted_average_reference([f.double() for f in flats], weights).float()
    torch.testing.assert_close(out, ref, atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("decoupled,wd", [(False, 0.0), (False, 0.01), (True, 0.1)])
def test_adam_step(decoupled, wd):
    n = 1 << 20
    torch.manual_seed(0)
    p = torch.randn(n, device="cuda")
    m = torch.zeros(n, device="cuda")
    v = torch.zeros(n, device="cuda")
    p_ref, m_ref, v_ref = p.clone(), m.clone(), v.clone()
    shadow = torch.empty(n, device="cuda", dtype=torch.bfloat16)
    for step in range(1, 4):
        g = torch.randn(n, device="cuda")
        ops.adam_step(p, g, m, v, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=wd, step=step, decoupled=decoupled, p_bf16=shadow)
        ops.adam_step_reference(p_ref, g, m_ref, v_ref, 1e-3, 0.9, 0.999, 1e-8, wd, step, decoupled)
    torch.testing.assert_close(p, p_ref, atol=1e-6, rtol=1e-5)
    torch.testing.assert_close(m, m_ref, atol=1e-6, rtol=1e-5)
    torch.testing.assert_close(v, v_ref, atol=1e-7, rtol=1e-5)
    torch.testing.assert_close(shadow, p.to(torch.bfloat16), atol=0, rtol=0)


@pytest.mark.parametrize("momentum,nesterov", [(0.0, False), (0.9, False), (0.9, True)])
def test_sgd_step(momentum, nesterov):
    n = 1 << 18
    torch.manual_seed(1)
    p = torch.randn(n, device="cuda")
    buf = torch.zeros(n, device="cuda") if momentum else None
    p_ref = p.clone()
    buf_ref = buf.clone() if buf is not None else None
    for step in range(3):
        g = torch.randn(n, device="cuda")
        ops.sgd_step(p, g, buf, lr=0.1, momentum=momentum, weight_decay=1e-4, nesterov=nesterov, first_step=step == 0)
        ops.sgd_step_reference(p_ref, g, buf_ref, 0.1, momentum, 0.0, 1e-4, nesterov, step == 0)
    torch.testing.assert_close(p, p_ref, atol=1e-6, rtol=1e-5)


def test_fedavg_uses_kernel_on_gpu():
    from collections import OrderedDict

    from p2pfl_amd.learning.aggregators import FedAvg
    from p2pfl_amd.learning.arena import flatten

    a = flatten(OrderedDict(w=torch.ones(100, device="cuda"), b=torch.zeros(3, device="cuda")))
    b = flatten(OrderedDict(w=torch.full((100,), 3.0, device="cuda"), b=torch.ones(3, device="cuda")))
    res = FedAvg().aggregate({"a": (a, 1), "b": (b, 3)})
    assert res.flat.is_cuda
    torch.testing.assert_close(res["w"], torch.full((100,), 2.5, device="cuda"))
    torch.testing.assert_close(res["b"], torch.full((3,), 0.75, device="cuda"))
