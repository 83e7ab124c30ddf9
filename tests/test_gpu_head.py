"""Pool + Linear + cross-entropy head (csrc/head.hip) vs fp32 PyTorch."""

from __future__ import annotations

import pytest
import torch
from torch import nn

from p2pfl_amd import ops
from p2pfl_amd.ops.head import head_ok, head_reference, head_xent

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B,C,H,W,N", [(32, 512, 4, 4, 10), (7, 2048, 4, 4, 10), (3, 64, 1, 1, 64), (70, 256, 2, 3, 5),
                                       (5, 20, 3, 3, 7), (4, 2048, 7, 7, 10)])
@pytest.mark.parametrize("wdtype", [torch.float32, torch.bfloat16])
def test_head_xent_vs_fp32(B, C, H, W, N, wdtype):
    ops.ext()
    g = torch.Generator(device="cuda").manual_seed(B + C + N)
    f = torch.randn(B, C, H, W, device="cuda", generator=g).to(torch.bfloat16)
    f = f.contiguous(memory_format=torch.channels_last).requires_grad_(True)
    fc = nn.Linear(C, N).cuda()
    fc.weight.data = fc.weight.data.to(wdtype)
    y = torch.randint(0, N, (B,), device="cuda", generator=g)
    assert head_ok(f, fc, y)
    loss, logits, acc = head_xent(f, fc, y)
    fr = f.detach().float().requires_grad_(True)
    wr = fc.weight.detach().float().requires_grad_(True)
    br = fc.bias.detach().float().requires_grad_(True)
    lr, logr = head_reference(fr, wr, br, y)
    torch.testing.assert_close(logits, logr, atol=1e-3, rtol=1e-3)
    torch.testing.assert_close(loss, lr, atol=1e-4, rtol=1e-4)
    assert abs(acc.item() - (logr.argmax(1) == y).float().mean().item()) < 1e-6
    loss.backward()
    lr.backward()
    torch.testing.assert_close(f.grad.float(), fr.grad, atol=1e-4, rtol=2e-2)
    tol = dict(atol=1e-3, rtol=1e-2) if wdtype == torch.bfloat16 else dict(atol=1e-5, rtol=1e-4)
    torch.testing.assert_close(fc.weight.grad.float(), wr.grad, **tol)
    torch.testing.assert_close(fc.bias.grad, br.grad, atol=1e-6, rtol=1e-4)
    assert fc.weight.grad.dtype == wdtype and f.grad.is_contiguous(memory_format=torch.channels_last)


def test_resnet_training_step_uses_native_head(monkeypatch):
    """ResNet's training step goes through the head kernels and matches the
    PyTorch head on the same features."""
    from p2pfl_amd.models.resnet import ResNet18

    ops.ext()
    m = ResNet18(seed=0).cuda().eval()
    x = torch.randint(0, 256, (4, 3, 32, 32), dtype=torch.uint8, device="cuda")
    y = torch.randint(0, 10, (4,), device="cuda")
    calls = []
    import p2pfl_amd.models.resnet as rn

    real = rn.head_xent
    monkeypatch.setattr(rn, "head_xent", lambda *a: calls.append(1) or real(*a))
    with torch.autocast("cuda", dtype=torch.bfloat16):
        f = m.features(x.float() / 255).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        loss = m.validation_step((x.float() / 255, y), 0)
    assert calls, "the head kernels did not run"
    lr, _ = head_reference(f, m.fc.weight, m.fc.bias, y)
    torch.testing.assert_close(loss, lr, atol=5e-3, rtol=5e-3)


def test_head_out_of_range_label_is_nan_not_clamped():
    """A label outside [0, N) gives a NaN loss and NaN gradients (F.cross_entropy
    raises): never the finite loss of a clamped label."""
    torch.manual_seed(0)
    f = torch.randn(4, 64, 4, 4, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    f.requires_grad_()
    fc = nn.Linear(64, 10).cuda()
    y = torch.tensor([1, 2, 10, 3], device="cuda")  # 10 is out of range
    assert head_ok(f, fc, y)
    loss, _, _ = head_xent(f, fc, y)
    assert torch.isnan(loss).item()
    loss.backward()
    assert torch.isnan(fc.weight.grad).any().item()
    y_neg = torch.tensor([1, 2, -100, 3], device="cuda")  # ignore_index is not supported either
    loss2, _, _ = head_xent(f.detach(), fc, y_neg)
    assert torch.isnan(loss2).item()


def test_resnet_with_custom_loss_fn_skips_the_native_head(monkeypatch):
    import p2pfl_amd.models.resnet as rn

    class Smoothed(rn.ResNet):
        def loss_fn(self, out, y):
            return nn.functional.cross_entropy(out, y, label_smoothing=0.1)

    ops.ext()
    m = Smoothed(rn.BasicBlock, [2, 2, 2, 2], 10, stem="cifar", seed=0).cuda()
    calls = []
    monkeypatch.setattr(rn, "head_xent", lambda *a: calls.append(1))
    x = torch.rand(2, 3, 32, 32, device="cuda")
    y = torch.randint(0, 10, (2,), device="cuda")
    with torch.autocast("cuda", dtype=torch.bfloat16):
        loss = m.training_step((x, y), 0)
    assert not calls and torch.isfinite(loss)


def test_head_weight_not_16_byte_aligned_takes_the_scalar_path():
    """A weight inside a shadow arena need not be 16-byte aligned: the launcher keeps the
    16-B vector path off there and the result still matches fp32."""
    ops.ext()
    B, C, H, W, N = 6, 1024, 4, 4, 10
    g = torch.Generator(device="cuda").manual_seed(11)
    f = torch.randn(B, C, H, W, device="cuda", generator=g).to(torch.bfloat16)
    f = f.contiguous(memory_format=torch.channels_last).requires_grad_(True)
    fc = nn.Linear(C, N).cuda()
    buf = torch.empty(N * C + 1, device="cuda", dtype=torch.bfloat16)
    buf[1:].copy_(fc.weight.detach().reshape(-1).to(torch.bfloat16))
    fc.weight.data = buf[1:].view(N, C)
    assert fc.weight.data_ptr() % 16 != 0
    y = torch.randint(0, N, (B,), device="cuda", generator=g)
    assert head_ok(f, fc, y)
    loss, logits, _ = head_xent(f, fc, y)
    fr = f.detach().float().requires_grad_(True)
    lr, logr = head_reference(fr, fc.weight.detach().float(), fc.bias.detach().float(), y)
    torch.testing.assert_close(logits, logr, atol=1e-3, rtol=1e-3)
    loss.backward()
    lr.backward()
    torch.testing.assert_close(f.grad.float(), fr.grad, atol=1e-4, rtol=2e-2)
