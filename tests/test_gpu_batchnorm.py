"""Fused BatchNorm(+residual)(+ReLU) HIP kernels vs fp32 PyTorch (MI355X only)."""

from __future__ import annotations

import pytest
import torch
from torch import nn

from p2pfl_amd import ops
from p2pfl_amd.ops.batchnorm import batch_norm_act, batch_norm_act_reference

pytestmark = pytest.mark.gpu


def _cl(t):
    return t.contiguous(memory_format=torch.channels_last)


def _bn(C, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    bn = nn.BatchNorm2d(C).cuda()
    with torch.no_grad():
        bn.weight.copy_(torch.rand(C, device="cuda", generator=g) + 0.5)
        bn.bias.copy_(torch.randn(C, device="cuda", generator=g))
        bn.running_mean.copy_(torch.randn(C, device="cuda", generator=g) * 0.1)
        bn.running_var.copy_(torch.rand(C, device="cuda", generator=g) + 0.5)
    return bn


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("shape", [(32, 64, 32, 32), (8, 512, 4, 4), (3, 96, 5, 7), (2, 2048, 2, 2), (2, 8, 1, 1)])
@pytest.mark.parametrize("residual,relu", [(False, True), (True, True), (False, False)])
def test_batch_norm_act_train(dtype, shape, residual, relu):
    ops.ext()
    g = torch.Generator(device="cuda").manual_seed(sum(shape))
    C = shape[1]
    x = _cl(torch.randn(*shape, device="cuda", generator=g) * 3 + 1.5).to(dtype).requires_grad_(True)
    r = _cl(torch.randn(*shape, device="cuda", generator=g)).to(dtype).requires_grad_(True) if residual else None
    bn = _bn(C, 7)
    ref = _bn(C, 7)
    y = batch_norm_act(x, bn, r, relu)
    assert y.dtype == dtype and y.shape == x.shape and y.is_contiguous(memory_format=torch.channels_last)
    xr = x.detach().float().requires_grad_(True)
    rr = r.detach().float().requires_grad_(True) if residual else None
    yr = batch_norm_act_reference(xr, ref.weight, ref.bias, ref.running_mean, ref.running_var, True, 0.1, ref.eps, rr, relu)
    tol = dict(atol=3e-2, rtol=2e-2) if dtype == torch.bfloat16 else dict(atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(y.float(), yr, **tol)
    # running statistics (unbiased variance) and the batch counter
    torch.testing.assert_close(bn.running_mean, ref.running_mean, atol=1e-5, rtol=1e-4)
    torch.testing.assert_close(bn.running_var, ref.running_var, atol=1e-5, rtol=1e-4)
    assert int(bn.num_batches_tracked) == 1
    # backward
    dy = _cl(torch.randn(*shape, device="cuda", generator=g)).to(dtype)
    y.backward(dy)
    yr.backward(dy.float())
    M = x.numel() // C
    grads = [(x.grad, xr.grad, "dx"), (bn.weight.grad, ref.weight.grad, "dw"), (bn.bias.grad, ref.bias.grad, "db")]
    if residual:
        grads.append((r.grad, rr.grad, "dres"))
    for a, e, name in grads:
        # relative to the gradient scale (dy ~ N(0, 1)); M = 2 makes dx ~ 0 exactly
        err = (a.float() - e.float()).abs().max().item() / max(e.float().abs().max().item(), 1.0)
        lim = (3e-2 if dtype == torch.bfloat16 else 1e-4) * (1 if name in ("dx", "dres") else max(1.0, (M / 4096) ** 0.5))
        assert err < lim, (name, err)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("residual", [False, True])
def test_batch_norm_act_eval(dtype, residual):
    g = torch.Generator(device="cuda").manual_seed(3)
    shape = (4, 128, 8, 8)
    x = _cl(torch.randn(*shape, device="cuda", generator=g)).to(dtype)
    r = _cl(torch.randn(*shape, device="cuda", generator=g)).to(dtype) if residual else None
    bn = _bn(128, 9).eval()
    with torch.no_grad():
        y = batch_norm_act(x, bn, r)
        yr = batch_norm_act_reference(x.float(), bn.weight, bn.bias, bn.running_mean, bn.running_var, False, 0.0, bn.eps, r.float() if residual else None)
    torch.testing.assert_close(y.float(), yr, **(dict(atol=3e-2, rtol=2e-2) if dtype == torch.bfloat16 else dict(atol=1e-5, rtol=1e-5)))


def test_batch_norm_is_deterministic():
    g = torch.Generator(device="cuda").manual_seed(5)
    x = _cl(torch.randn(16, 256, 16, 16, device="cuda", generator=g)).to(torch.bfloat16)
    dy = _cl(torch.randn(16, 256, 16, 16, device="cuda", generator=g)).to(torch.bfloat16)
    outs = []
    for _ in range(2):
        bn = _bn(256, 1)
        xi = x.clone().requires_grad_(True)
        y = batch_norm_act(xi, bn)
        y.backward(dy)
        outs.append((y, xi.grad, bn.weight.grad, bn.bias.grad, bn.running_var.clone()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_batch_norm_large_mean_no_cancellation():
    """Shifted sums keep the variance exact for activations far from zero."""
    g = torch.Generator(device="cuda").manual_seed(11)
    x = _cl(torch.randn(8, 64, 16, 16, device="cuda", generator=g) * 0.01 + 300.0)
    bn = _bn(64, 2)
    ref = _bn(64, 2)
    y = batch_norm_act(x, bn, relu=False)
    yr = batch_norm_act_reference(x.double(), ref.weight.double(), ref.bias.double(), ref.running_mean.double(), ref.running_var.double(), True, 0.1, ref.eps, None, False)
    torch.testing.assert_close(y.double(), yr, atol=2e-3, rtol=1e-3)


def test_resnet18_uses_fused_bn_and_trains():
    from p2pfl_amd.models.resnet import ResNet18

    torch.manual_seed(0)
    m = ResNet18(seed=0).cuda()
    x = torch.randint(0, 255, (16, 3, 32, 32), dtype=torch.uint8, device="cuda")
    y = torch.randint(0, 10, (16,), device="cuda")
    calls = {"n": 0}
    real = ops.ext().bn.fwd_train
    import p2pfl_amd.ops.batchnorm as bnmod

    orig = bnmod._bx

    def spy():
        b = orig()

        class W:
            def fwd_train(self, *a, **k):
                calls["n"] += 1
                return real(*a, **k)

            def __getattr__(self, k):
                return getattr(b, k)

        return W()

    bnmod._bx = spy
    try:
        opt = torch.optim.SGD(m.parameters(), lr=0.05, momentum=0.9)
        losses = []
        for _ in range(15):
            opt.zero_grad()
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = torch.nn.functional.cross_entropy(m(x), y)
            loss.backward()
            opt.step()
            losses.append(float(loss))
    finally:
        bnmod._bx = orig
    assert calls["n"] == 15 * 20, calls  # stem + 16 block BNs + 3 projection BNs per step
    assert losses[-1] < 0.5 * losses[0], losses
    # eval forward agrees with the PyTorch chain
    m.eval()
    import os

    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        a = m(x).float()
        os.environ["P2PFL_FORCE_TORCH_OPS"] = "1"
        try:
            b = m(x).float()
        finally:
            del os.environ["P2PFL_FORCE_TORCH_OPS"]
    torch.testing.assert_close(a, b, atol=0.15, rtol=0.05)


@pytest.mark.parametrize("shape", [(32, 64, 32, 32), (5, 64, 9, 11), (8, 512, 4, 4), (2, 2048, 2, 2), (3, 24, 5, 7)])
@pytest.mark.parametrize("residual,relu", [(False, True), (True, False)])
def test_fused_stats_finalize_matches_separate_launches(shape, residual, relu):
    """Statistics + finalize in one launch (last block to arrive finalizes) vs the
    separate statistics / finalize launches: same values up to the reduction order,
    and the arrival counter is zero again after each launch."""
    bx = ops.ext().bn
    C = shape[1]
    M = shape[0] * shape[2] * shape[3]
    assert bx.fused_rows(M, C) > 0
    g = torch.Generator(device="cuda").manual_seed(M + C)
    x = torch.randn(M, C, device="cuda", generator=g).mul(2).add(0.5).to(torch.bfloat16)
    r = torch.randn(M, C, device="cuda", generator=g).to(torch.bfloat16) if residual else None
    dy = torch.randn(M, C, device="cuda", generator=g).to(torch.bfloat16)
    outs = []
    for fused in (True, False):
        bn = _bn(C, 4)
        ctr = torch.zeros(16, dtype=torch.int32, device="cuda") if fused else None
        y, mean, rstd = bx.fwd_train(x, bn.weight, bn.bias, r, bn.running_mean, bn.running_var, bn.num_batches_tracked,
                                     0.1, 1e-5, relu, ctr)
        back = bx.bwd(dy, y, x, bn.weight, mean, rstd, relu, residual, ctr)
        torch.cuda.synchronize()
        if fused:
            assert int(ctr.abs().sum()) == 0
        outs.append((y.float(), mean, rstd, bn.running_mean.clone(), bn.running_var.clone(), int(bn.num_batches_tracked),
                     *[t.float() for t in back]))
    (yf, *rest_f), (ys, *rest_s) = outs
    torch.testing.assert_close(yf, ys, atol=2e-2, rtol=1e-2)
    for a, b in zip(rest_f, rest_s):
        if isinstance(a, int):
            assert a == b == 1
        elif a.dtype == torch.float32 and a.dim() == 1:
            torch.testing.assert_close(a, b, atol=1e-4, rtol=1e-4)
        else:
            torch.testing.assert_close(a, b, atol=2e-2, rtol=1e-2)


# ---- convolution launch computing the BatchNorm statistics (gemm_core.h BnEpi) -------------
CONV_BN_CASES = [
    # N, C, H, W, O, stride: tiles_m 256 (16 groups), 2 tile columns, ragged rows, split-K shapes
    (32, 64, 32, 32, 64, 1),
    (8, 64, 16, 16, 256, 2),
    (3, 128, 7, 5, 128, 1),
    (32, 256, 4, 4, 512, 1),
    (2, 64, 33, 9, 64, 1),
]


@pytest.mark.parametrize("N,C,H,W,O,s", CONV_BN_CASES)
@pytest.mark.parametrize("residual,relu", [(False, True), (True, True), (False, False)])
def test_conv_bn_act_statistics_epilogue_vs_fp32(monkeypatch, N, C, H, W, O, s, residual, relu):
    """conv_bn_act: the convolution launch computes batch mean / variance of its bf16 output,
    the apply coefficients and the running statistics; output, running stats and all
    gradients match conv + BatchNorm (+ residual) (+ ReLU) in fp32 on the same bf16 operands."""
    from p2pfl_amd.ops import conv as conv_ops
    import torch.nn.functional as F

    ops.ext()
    monkeypatch.setattr(conv_ops, "_POLICY", "native")
    monkeypatch.setattr(conv_ops, "_FUSED_BN", True)  # the epilogue under test (off by default: slower)
    g = torch.Generator(device="cuda").manual_seed(N * 7 + O)
    x = _cl(torch.randn(N, C, H, W, device="cuda", generator=g)).to(torch.bfloat16).requires_grad_(True)
    conv = nn.Conv2d(C, O, 3, s, 1, bias=False).cuda()
    with torch.no_grad():
        conv.weight.copy_(torch.randn(O, C, 3, 3, device="cuda", generator=g) / (9 * C) ** 0.5 + 0.02)
    conv.weight.data = conv.weight.data.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    bn, ref = _bn(O, 11), _bn(O, 11)
    OH, OW = (H + 2 - 3) // s + 1, (W + 2 - 3) // s + 1
    r = _cl(torch.randn(N, O, OH, OW, device="cuda", generator=g)).to(torch.bfloat16).requires_grad_(True) if residual else None
    before = conv_ops.STATS["native_fwd_bn"]
    y = conv_ops.conv_bn_act(x, conv, bn, r, relu)
    assert conv_ops.STATS["native_fwd_bn"] == before + 1
    xr = x.detach().float().requires_grad_(True)
    wr = conv.weight.detach().float().requires_grad_(True)
    rr = r.detach().float().requires_grad_(True) if residual else None
    yc = F.conv2d(xr, wr, None, s, 1)
    # the kernel normalises its bf16-rounded output: the reference does the same
    yc_b = yc + (yc.detach().to(torch.bfloat16).float() - yc.detach())
    yr = batch_norm_act_reference(yc_b, ref.weight, ref.bias, ref.running_mean, ref.running_var, True, 0.1, ref.eps, rr, relu)
    torch.testing.assert_close(y.float(), yr, atol=4e-2, rtol=2e-2)
    torch.testing.assert_close(bn.running_mean, ref.running_mean, atol=1e-4, rtol=1e-3)
    torch.testing.assert_close(bn.running_var, ref.running_var, atol=1e-4, rtol=1e-3)
    assert int(bn.num_batches_tracked) == 1
    dy = _cl(torch.randn(y.shape, device="cuda", generator=g)).to(torch.bfloat16)
    y.backward(dy)
    yr.backward(dy.float())
    for a, e, name in [(x.grad, xr.grad, "dx"), (conv.weight.grad, wr.grad, "dW"), (bn.weight.grad, ref.weight.grad, "dgamma"),
                       (bn.bias.grad, ref.bias.grad, "dbeta")] + ([(r.grad, rr.grad, "dres")] if residual else []):
        scale = e.abs().max().item() + 1e-6
        torch.testing.assert_close(a.float(), e, atol=3e-2 * scale, rtol=3e-2, msg=lambda m, n=name: f"{n}: {m}")


def test_conv_bn_statistics_are_deterministic_and_counters_reset(monkeypatch):
    """Repeated launches (counters reused from the ring) give bitwise-equal statistics."""
    from p2pfl_amd.ops import conv as conv_ops

    ops.ext()
    monkeypatch.setattr(conv_ops, "_FUSED_BN", True)
    monkeypatch.setattr(conv_ops, "_POLICY", "native")
    x = _cl(torch.randn(32, 64, 32, 32, device="cuda")).to(torch.bfloat16)
    conv = nn.Conv2d(64, 64, 3, 1, 1, bias=False).cuda()
    conv.weight.data = conv.weight.data.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    outs = []
    for _ in range(4):
        bn = _bn(64, 3)
        with torch.no_grad():
            outs.append((conv_ops.conv_bn_act(x, conv, bn), bn.running_mean.clone(), bn.running_var.clone()))
    for o in outs[1:]:
        for a, b in zip(outs[0], o):
            assert torch.equal(a, b)


@pytest.mark.parametrize("block,cin,cout,stride,hw", [("basic", 64, 64, 1, 16), ("basic", 64, 128, 2, 16),
                                                       ("bottleneck", 256, 64, 1, 8), ("bottleneck", 64, 128, 2, 8)])
def test_fused_block_chain_matches_separate_bn_kernels_and_fp32(monkeypatch, block, cin, cout, stride, hw):
    """A whole ResNet block on the fused chain (conv launches computing BN statistics,
    the inner convolutions' input-gradient launches computing the previous BN's backward
    statistics) against (a) the same bf16 block with the separate BN kernels and (b) the
    block in fp32 PyTorch: output, running statistics, input gradient and every
    parameter gradient."""
    import copy

    from p2pfl_amd.models.resnet import BasicBlock, Bottleneck, _pair
    from p2pfl_amd.ops import conv as conv_ops

    ops.ext()
    monkeypatch.setattr(conv_ops, "_POLICY", "native")

    def _blk(m, x):  # blocks return a forked (conv input, shortcut input) pair
        return _pair(m(x))[0]
    torch.manual_seed(cin + cout + stride)
    blk = (BasicBlock(cin, cout, stride) if block == "basic" else Bottleneck(cin, cout, stride)).cuda().train()
    ref = copy.deepcopy(blk).float()
    for m in blk.modules():
        if isinstance(m, nn.Conv2d):
            m.weight.data = m.weight.data.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    sep = copy.deepcopy(blk)
    for m in ref.modules():
        if isinstance(m, nn.Conv2d):
            m.weight.data = m.weight.data.to(torch.bfloat16).float()
    x0 = _cl(torch.randn(16, cin, hw, hw, device="cuda")).to(torch.bfloat16)
    dy = _cl(torch.randn(_blk(blk, x0.clone()).shape, device="cuda")).to(torch.bfloat16)
    for m in (blk, sep):  # the probe call above advanced blk's running statistics: start both fresh
        for b in m.modules():
            if isinstance(b, nn.BatchNorm2d):
                b.reset_running_stats()
    for b in ref.modules():
        if isinstance(b, nn.BatchNorm2d):
            b.reset_running_stats()

    def run(model, fused):
        monkeypatch.setattr(conv_ops, "_FUSED_BN", fused)
        x = x0.clone().requires_grad_(True)
        before = conv_ops.STATS["bn_act_conv"]
        y = _blk(model, x)
        assert (conv_ops.STATS["bn_act_conv"] > before) == fused
        y.backward(dy)
        return x, y

    xf, yf = run(blk, True)
    xs, ys = run(sep, False)
    xr = x0.float().requires_grad_(True)
    yr = _blk(ref, xr)
    yr.backward(dy.float())

    def rel(a, e):
        return ((a.float() - e.float()).norm() / (e.float().norm() + 1e-12)).item()

    # (a) fused vs separate BN kernels: same bf16 arithmetic up to summation order
    assert rel(yf, ys) < 1e-2
    for (n, a), b in zip(blk.named_buffers(), sep.buffers()):
        if a.dtype.is_floating_point:
            torch.testing.assert_close(a, b, atol=1e-3, rtol=1e-2, msg=lambda m, n=n: f"{n}: {m}")
        else:
            assert torch.equal(a, b), n
    pairs = [("x", xf.grad, xs.grad, xr.grad)] + [
        (n, a.grad, b.grad, c.grad) for (n, a), b, c in zip(blk.named_parameters(), sep.parameters(), ref.parameters())]
    for n, a, b, c in pairs:
        assert a is not None and b is not None, n
        assert rel(a, b) < 3e-2, f"{n}: fused vs separate BN kernels, relative L2 error {rel(a, b):.3g}"
        # (b) vs fp32: bf16 activations flip a few ReLU masks; a loose sanity bound
        assert rel(a, c) < 0.12, f"{n}: fused vs fp32, relative L2 error {rel(a, c):.3g}"
    torch.testing.assert_close(yf.float(), yr, atol=8e-2, rtol=5e-2)


@pytest.mark.parametrize("block", ["basic", "bottleneck"])
def test_forked_block_inputs_sum_gradients_in_bn_kernels(monkeypatch, block):
    """Two blocks in a row: the first block's output BN forks (conv input, shortcut input)
    and the second block's two branch gradients are summed inside that BN's backward
    kernels (dy2) -- same output and gradients as one output with autograd's add."""
    import copy

    from p2pfl_amd.models import resnet as rn
    from p2pfl_amd.ops import batchnorm as bn_ops
    from p2pfl_amd.ops import conv as conv_ops

    ops.ext()
    monkeypatch.setattr(conv_ops, "_POLICY", "native")
    torch.manual_seed(3)
    mk = (lambda: rn.BasicBlock(64, 64, 1)) if block == "basic" else (lambda: rn.Bottleneck(256, 64, 1))
    net = nn.Sequential(mk(), mk()).cuda().train()
    for m in net.modules():
        if isinstance(m, nn.Conv2d):
            m.weight.data = m.weight.data.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    twin = copy.deepcopy(net)
    cin = 64 if block == "basic" else 256
    x0 = _cl(torch.randn(8, cin, 16, 16, device="cuda")).to(torch.bfloat16)
    dy = _cl(torch.randn(8, cin, 16, 16, device="cuda")).to(torch.bfloat16)

    def run(model, fork):
        monkeypatch.setattr(rn, "_FORK", fork)
        x = x0.clone().requires_grad_(True)
        before = bn_ops.STATS["dy_pairs"]
        y = rn._pair(model(x))[0]
        y.backward(dy)
        assert (bn_ops.STATS["dy_pairs"] > before) == fork
        return x, y

    xf, yf = run(net, True)
    xu, yu = run(twin, False)
    torch.testing.assert_close(yf.float(), yu.float(), atol=0, rtol=0)

    def rel(a, e):  # relative norm: the two runs differ only in where the branch sum is rounded to bf16
        return ((a.float() - e.float()).norm() / (e.float().norm() + 1e-12)).item()

    assert rel(xf.grad, xu.grad) < 1e-2
    for (n, a), b in zip(net.named_parameters(), twin.parameters()):
        assert rel(a.grad, b.grad) < 2e-2, (n, rel(a.grad, b.grad))
