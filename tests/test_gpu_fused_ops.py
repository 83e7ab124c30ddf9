"""Fused LayerNorm / bias+GELU / softmax cross-entropy HIP kernels vs fp32 PyTorch (MI355X only)."""

from __future__ import annotations

import pytest
import torch

from p2pfl_amd import ops

pytestmark = pytest.mark.gpu


def _inputs(shape, dtype, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return (torch.randn(*shape, device="cuda", generator=g) * 2 + 0.5).to(dtype)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("N,C", [(394, 768), (7, 192), (33, 1024), (5, 2048), (3, 24)])
def test_layer_norm_fwd_bwd(dtype, N, C):
    ops.ext()
    x = _inputs((N, C), dtype, C).requires_grad_(True)
    w = (torch.rand(C, device="cuda") + 0.5).requires_grad_(True)
    b = torch.randn(C, device="cuda").requires_grad_(True)
    y = ops.layer_norm(x, w, b, 1e-6)
    assert y.dtype == dtype
    xr = x.detach().float().requires_grad_(True)
    wr, br = w.detach().clone().requires_grad_(True), b.detach().clone().requires_grad_(True)
    yr = ops.layer_norm_reference(xr, wr, br, 1e-6)
    tol = dict(atol=2e-2, rtol=2e-2) if dtype == torch.bfloat16 else dict(atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(y.float(), yr, **tol)
    dy = _inputs((N, C), dtype, C + 1)
    y.backward(dy)
    yr.backward(dy.float())
    torch.testing.assert_close(x.grad.float(), xr.grad, **(dict(atol=3e-2, rtol=3e-2) if dtype == torch.bfloat16 else dict(atol=1e-4, rtol=1e-4)))
    torch.testing.assert_close(w.grad, wr.grad, atol=1e-3 * N, rtol=1e-3)
    torch.testing.assert_close(b.grad, br.grad, atol=1e-3 * N, rtol=1e-3)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("shape", [(2, 197, 3072), (37, 128), (1, 8)])
def test_bias_gelu_fwd_bwd(dtype, shape):
    ops.ext()
    H = shape[-1]
    x = _inputs(shape, dtype, 3).requires_grad_(True)
    b = torch.randn(H, device="cuda").requires_grad_(True)
    y = ops.bias_gelu(x, b)
    xr = x.detach().float().requires_grad_(True)
    br = b.detach().clone().requires_grad_(True)
    yr = ops.bias_gelu_reference(xr, br)
    tol = dict(atol=1e-2, rtol=1e-2) if dtype == torch.bfloat16 else dict(atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(y.float(), yr, **tol)
    dy = _inputs(shape, dtype, 4)
    y.backward(dy)
    yr.backward(dy.float())
    torch.testing.assert_close(x.grad.float(), xr.grad, **tol)
    n = x.numel() // H
    torch.testing.assert_close(b.grad, br.grad, atol=2e-2 * max(1, n) ** 0.5 if dtype == torch.bfloat16 else 1e-4, rtol=2e-2)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("N,K", [(64, 10), (13, 1000), (1, 3)])
def test_softmax_xent_fwd_bwd(dtype, N, K):
    ops.ext()
    z = _inputs((N, K), dtype, K).requires_grad_(True)
    y = torch.randint(0, K, (N,), device="cuda")
    loss = ops.softmax_xent(z, y)
    zr = z.detach().float().requires_grad_(True)
    lr_ = ops.softmax_xent_reference(zr, y)
    torch.testing.assert_close(loss, lr_, atol=1e-4, rtol=1e-4)
    (3.0 * loss).backward()
    (3.0 * lr_).backward()
    tol = dict(atol=2e-3, rtol=2e-2) if dtype == torch.bfloat16 else dict(atol=1e-6, rtol=1e-5)
    torch.testing.assert_close(z.grad.float(), zr.grad, **tol)


def test_vit_uses_fused_kernels_and_trains():
    from p2pfl_amd.models.vit import ViT_Tiny

    torch.manual_seed(0)
    m = ViT_Tiny(seed=0).cuda()
    x = torch.randint(0, 255, (16, 3, 32, 32), dtype=torch.uint8, device="cuda")
    y = torch.randint(0, 10, (16,), device="cuda")
    opt = torch.optim.AdamW(m.parameters(), lr=1e-3)
    losses = []
    for _ in range(40):
        opt.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = m.loss_fn(m(x), y)
        loss.backward()
        opt.step()
        losses.append(float(loss))
    assert losses[-1] < 0.8 * losses[0], losses
    # the same model in fp32 PyTorch agrees on the first forward
    ref = ViT_Tiny(seed=0).cuda()
    with torch.no_grad():
        import os

        os.environ["P2PFL_FORCE_TORCH_OPS"] = "1"
        try:
            a = ref(x)
        finally:
            del os.environ["P2PFL_FORCE_TORCH_OPS"]
        b = ViT_Tiny(seed=0).cuda()(x)
    torch.testing.assert_close(a, b, atol=1e-3, rtol=1e-3)


def test_vit_class_token_only_last_block_matches_full(monkeypatch):
    """The fused encoder's last block after its attention on the class-token rows only:
    the same logits and parameter gradients as running it over every token."""
    from p2pfl_amd.models import vit

    x = torch.randint(0, 255, (8, 3, 32, 32), dtype=torch.uint8, device="cuda")
    y = torch.randint(0, 10, (8,), device="cuda")
    outs = []
    for cls_only in (False, True):
        monkeypatch.setattr(vit, "_CLS_ONLY", cls_only)
        m = vit.ViT_Tiny(seed=0).cuda()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            z = m(x)
            loss = m.loss_fn(z, y)
        loss.backward()
        outs.append((z.float(), {n: p.grad.float() for n, p in m.named_parameters()}))
    (za, ga), (zb, gb) = outs
    torch.testing.assert_close(zb, za, atol=2e-2, rtol=2e-2)
    for n in ga:
        torch.testing.assert_close(gb[n], ga[n], atol=2e-3, rtol=5e-2, msg=lambda m: f"{n}: {m}")


def test_linear_gelu_eval_forward_without_pre_activation():
    """Under no_grad the GELU epilogue skips the pre-activation store; the output is the
    training forward's, bit for bit (same tuned kernel configuration)."""
    torch.manual_seed(3)
    x = torch.randn(512, 256, device="cuda").to(torch.bfloat16)
    w = (torch.randn(1024, 256, device="cuda") * 0.05).requires_grad_(True)
    b = torch.randn(1024, device="cuda").requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        yt = ops.linear_gelu(x, w, b)
        with torch.no_grad():
            ye = ops.linear_gelu(x, w, b)
    assert yt.requires_grad and not ye.requires_grad
    assert torch.equal(yt.detach(), ye)
    ref = torch.nn.functional.gelu(x.float() @ w.detach().to(torch.bfloat16).float().t() + b.detach())
    torch.testing.assert_close(ye.float(), ref, atol=3e-2, rtol=2e-2)


@pytest.mark.parametrize("B,T,H", [(2, 197, 12), (3, 65, 3), (1, 1, 2), (2, 32, 1), (1, 256, 2), (2, 100, 4)])
def test_attention_fwd_bwd(B, T, H):
    """Fused MHSA kernel vs fp32 SDPA on the same bf16 inputs (forward, dq/dk/dv)."""
    torch.manual_seed(B * 1000 + T + H)
    C = 64 * H
    qkv = (torch.randn(B, T, 3 * C, device="cuda") * 1.5).to(torch.bfloat16).requires_grad_(True)
    ref_in = qkv.detach().float().requires_grad_(True)
    y = ops.attention_qkv(qkv, H)
    ref = ops.attention_qkv_reference(ref_in, H)
    assert y.dtype == torch.bfloat16 and y.shape == (B, T, C)
    torch.testing.assert_close(y.float(), ref, atol=2e-2, rtol=2e-2)
    g = torch.randn(B, T, C, device="cuda").to(torch.bfloat16)
    y.backward(g)
    ref.backward(g.float())
    d, dr = qkv.grad.float(), ref_in.grad
    for part, name in enumerate("qkv"):
        a, b = d[..., part * C:(part + 1) * C], dr[..., part * C:(part + 1) * C]
        err = (a - b).abs().max().item() / max(b.abs().max().item(), 1e-6)
        assert err < 3e-2, (name, err)


def test_attention_rejects_unsupported_shapes():
    qkv = torch.zeros(1, 300, 3 * 64, device="cuda", dtype=torch.bfloat16)
    with pytest.raises(RuntimeError):
        ops.ext().fused.attn_fwd(qkv, 1)  # T > 256
    with pytest.raises(RuntimeError):
        ops.ext().fused.attn_fwd(torch.zeros(1, 8, 3 * 96, device="cuda", dtype=torch.bfloat16), 1)  # head dim 96
    # the Python entry point falls back to SDPA for such shapes
    y = ops.attention_qkv(torch.randn(1, 300, 3 * 64, device="cuda", dtype=torch.bfloat16), 1)
    assert y.shape == (1, 300, 64)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("N,C", [(394, 768), (7, 192), (33, 1024)])
def test_add_layer_norm_fwd_bwd(dtype, N, C):
    """Fused residual add + LayerNorm vs separate add then fp32 LayerNorm."""
    x = _inputs((N, C), dtype, 11).requires_grad_(True)
    r = _inputs((N, C), dtype, 12).requires_grad_(True)
    w = (torch.rand(C, device="cuda") + 0.5).requires_grad_(True)
    b = torch.randn(C, device="cuda").requires_grad_(True)
    s, y = ops.add_layer_norm(x, r, w, b, 1e-6)
    xr, rr = x.detach().clone().requires_grad_(True), r.detach().clone().requires_grad_(True)
    wr, br = w.detach().clone().requires_grad_(True), b.detach().clone().requires_grad_(True)
    sr = (xr + rr).to(dtype)
    yr = torch.nn.functional.layer_norm(sr.float(), (C,), wr, br, 1e-6)
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-4
    torch.testing.assert_close(s, sr, atol=0, rtol=0)
    torch.testing.assert_close(y.float(), yr, atol=tol * 4, rtol=tol)
    gs, gy = _inputs((N, C), dtype, 13), _inputs((N, C), dtype, 14)
    torch.autograd.backward([s, y], [gs, gy])
    torch.autograd.backward([sr, yr], [gs, gy.float()])
    for a, e in ((x.grad, xr.grad), (r.grad, rr.grad), (w.grad, wr.grad), (b.grad, br.grad)):
        err = (a.float() - e.float()).abs().max().item() / max(e.float().abs().max().item(), 1e-6)
        assert err < (3e-2 if dtype == torch.bfloat16 else 1e-4), err


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_linear_fused_bias_grad(dtype):
    torch.manual_seed(5)
    x = torch.randn(4, 197, 768, device="cuda", dtype=dtype, requires_grad=True)
    w = (torch.randn(2304, 768, device="cuda") * 0.02).to(dtype).requires_grad_(True)
    b = torch.randn(2304, device="cuda", dtype=dtype, requires_grad=True)
    y = ops.linear(x, w, b)
    ref = torch.nn.functional.linear(x.detach().float().requires_grad_(True), w.detach().float().requires_grad_(True), b.detach().float().requires_grad_(True))
    torch.testing.assert_close(y.float(), ref, atol=5e-2, rtol=2e-2)
    g = torch.randn_like(y)
    y.backward(g)
    col = g.float().reshape(-1, 2304).sum(0)
    torch.testing.assert_close(b.grad.float(), col, atol=1e-1 if dtype == torch.bfloat16 else 1e-3, rtol=1e-2)
    torch.testing.assert_close(ops.ext().fused.column_sum(g.reshape(-1, 2304).contiguous()), col, atol=1e-2, rtol=1e-4)


@pytest.mark.parametrize("N,K", [(768, 768), (2304, 768), (768, 3072)])
def test_linear_split_k_weight_grad(N, K):
    """ViT-sized weight gradients take the split-K bmm path; compare with an fp32 reference."""
    from p2pfl_amd.ops.fused import _wgrad_splits

    M = 32 * 197
    assert _wgrad_splits(M, N, K) > 1
    torch.manual_seed(N + K)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    w = (torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16).requires_grad_(True)
    b = torch.zeros(N, device="cuda", requires_grad=True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = ops.linear(x, w, b)
    g = torch.randn_like(y)
    y.backward(g)
    ref = g.float().t() @ x.detach().float()
    err = (w.grad.float() - ref).abs().max().item() / ref.abs().max().item()
    assert w.grad.dtype == torch.bfloat16 and err < 1e-2, err


def test_split_sum_and_bf16_column_sum():
    """Split-K partial reduction and the bf16-out column sum == fp32 PyTorch sums rounded to bf16."""
    torch.manual_seed(4)
    for S, shape in ((2, (768, 2304)), (4, (3072, 768)), (3, (8, 40))):
        parts = torch.randn(S, *shape, device="cuda").to(torch.bfloat16)
        want = parts.float().sum(0).to(torch.bfloat16)
        got = ops.ext().fused.split_sum_bf16(parts)
        assert got.shape == want.shape and got.dtype == torch.bfloat16
        torch.testing.assert_close(got.float(), want.float(), atol=0, rtol=1e-2)
        assert (got != want).float().mean() < 1e-3  # fp32 summation order only
    g = torch.randn(6304, 768, device="cuda").to(torch.bfloat16)
    f32 = ops.ext().fused.column_sum(g)
    b16 = ops.ext().fused.column_sum(g, True)
    assert b16.dtype == torch.bfloat16 and torch.equal(b16, f32.to(torch.bfloat16))
    torch.testing.assert_close(f32, g.float().sum(0), atol=1e-2, rtol=1e-4)


def test_patchify_u8_matches_the_eager_prologue():
    """One kernel: the same bf16 patch rows as float cast, /255, patch permute and the
    GEMM's bf16 cast (bitwise)."""
    from p2pfl_amd import ops as O

    O.ext()
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.randint(0, 256, (3, 3, 32, 48), dtype=torch.uint8, device="cuda", generator=g)
    P = 16
    xf = x.float().mul_(1.0 / 255.0)
    B, C, H, W = x.shape
    want = xf.view(B, C, H // P, P, W // P, P).permute(0, 2, 4, 1, 3, 5).reshape(B, (H // P) * (W // P), C * P * P)
    got = O.patchify_u8(x, P)
    assert got.dtype == torch.bfloat16 and got.shape == want.shape
    assert torch.equal(got, want.to(torch.bfloat16))


@pytest.mark.parametrize("B,N,D", [(4, 196, 768), (3, 5, 64)])
def test_embed_tokens_fwd_bwd(B, N, D):
    """cat(cls, y) + pos and its backward (patch-token gradient, batch sums for pos / cls)
    against the torch composition on the same bf16 operands."""
    from p2pfl_amd import ops as O

    O.ext()
    g = torch.Generator(device="cuda").manual_seed(B + N)
    y = torch.randn(B, N, D, device="cuda", generator=g).to(torch.bfloat16).requires_grad_()
    cls = (torch.randn(1, 1, D, device="cuda", generator=g) * 0.02).to(torch.bfloat16).requires_grad_()
    pos = (torch.randn(1, N + 1, D, device="cuda", generator=g) * 0.02).to(torch.bfloat16).requires_grad_()
    h = O.embed_tokens(y, cls, pos)
    ref = torch.cat([cls.expand(B, -1, -1), y], dim=1) + pos
    assert torch.equal(h, ref)
    dh = torch.randn(B, N + 1, D, device="cuda", generator=g).to(torch.bfloat16)
    gy, gc, gp = torch.autograd.grad(h, (y, cls, pos), dh)
    ry, rc, rp = torch.autograd.grad(ref, (y, cls, pos), dh)
    assert torch.equal(gy, ry)
    assert gc.shape == rc.shape and gp.shape == rp.shape
    torch.testing.assert_close(gp.float(), dh.float().sum(0, keepdim=True), atol=2e-2, rtol=1e-2)
    torch.testing.assert_close(gc.float(), dh[:, :1].float().sum(0, keepdim=True), atol=2e-2, rtol=1e-2)


def test_deferred_param_grad_reductions_are_bitwise_equal():
    """ops.fused.deferred_param_grads: the LayerNorm / bias gradients reduced in one
    col_reduce_multi launch after the backward equal the per-pass reductions bit for bit."""
    from p2pfl_amd.models.vit import ViT_Tiny
    from p2pfl_amd.ops import fused

    x = torch.randint(0, 255, (8, 3, 32, 32), dtype=torch.uint8, device="cuda")
    y = torch.randint(0, 10, (8,), device="cuda")
    grads = []
    for defer in (False, False, True):  # the first pass tunes every product's kernel
        m = ViT_Tiny(seed=0).cuda()
        with fused.deferred_param_grads(enabled=defer):
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = m.loss_fn(m(x), y)
            loss.backward()
        grads.append({n: p.grad.clone() for n, p in m.named_parameters()})
    ref, got = grads[1], grads[2]
    assert ref.keys() == got.keys()
    for n in ref:
        assert got[n].dtype == ref[n].dtype and torch.equal(got[n], ref[n]), n


def test_col_reduce_multi_vs_torch():
    """More jobs than one launch's table (40): fp32 and bf16 outputs vs fp64 column sums."""
    torch.manual_seed(5)
    parts, outs, refs = [], [], []
    for i in range(45):
        R, C = 1 + (i * 37) % 300, 8 * (1 + (i * 13) % 97)
        p = torch.randn(R, C, device="cuda")
        parts.append(p)
        outs.append(torch.empty(C, device="cuda", dtype=torch.bfloat16 if i % 3 == 0 else torch.float32))
        refs.append(p.double().sum(0))
    ops.ext().fused.col_reduce_multi(parts, outs)
    for o, r in zip(outs, refs):
        tol = dict(atol=2e-2, rtol=1e-2) if o.dtype == torch.bfloat16 else dict(atol=1e-4, rtol=1e-5)
        torch.testing.assert_close(o.double(), r, **tol)


def test_column_sum_parts_multi_bitwise_equals_column_sum():
    """More activations than one launch's table (64): the batched partials + batched
    reduction give exactly column_sum's fp32 / bf16 results."""
    fx = ops.ext().fused
    torch.manual_seed(6)
    xs = [torch.randn(1 + (i * 97) % 700, 8 * (1 + (i * 29) % 130), device="cuda").to(torch.bfloat16) for i in range(70)]
    parts = [torch.empty(fx.colsum_splits(x.shape[0]), x.shape[1], device="cuda") for x in xs]
    fx.column_sum_parts_multi(xs, parts)
    outs = [torch.empty(x.shape[1], device="cuda", dtype=torch.bfloat16 if i % 2 else torch.float32)
            for i, x in enumerate(xs)]
    fx.col_reduce_multi(parts, outs)
    for i, (x, o) in enumerate(zip(xs, outs)):
        assert torch.equal(o, fx.column_sum(x, bool(i % 2))), i
