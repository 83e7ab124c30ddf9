"""Per-kernel numerics of the fused CNN step (MI355X only).

Each HIP kernel gets exactly the bf16 inputs it sees in training and is
compared against a plain PyTorch fp32 implementation of the same op computed
from those same inputs, so bf16 storage of activations is the only expected
difference (plus fp32 summation order).
"""

from __future__ import annotations

import pytest
import torch
import torch.nn.functional as F

from p2pfl_amd import ops
from p2pfl_amd.models import CNN

pytestmark = pytest.mark.gpu

B = 32


@pytest.fixture(scope="module")
def eng():
    from p2pfl_amd.learning.fused_cnn import FusedCNNEngine

    ops.ext()
    torch.manual_seed(0)
    return FusedCNNEngine(CNN(seed=3).cuda(), device=torch.device("cuda"))


def _p(eng, name):
    return eng.arena.params[name]


def _bf(t):
    return t.to(torch.bfloat16).float()


def _close(got, want, rtol=1e-2, atol=1e-3):
    err = (got.float() - want.float()).abs()
    bound = atol + rtol * want.float().abs()
    frac = float((err > bound).float().mean())
    return frac


def _forward(eng, x, train=False, nb=B):
    from p2pfl_amd.learning import fused_cnn

    stats = torch.zeros(4, device="cuda")
    y = torch.zeros(nb, dtype=torch.int64, device="cuda")
    old = fused_cnn._CONV12
    fused_cnn._CONV12 = False  # the per-kernel tests read P1, which only the two-kernel path writes
    try:
        eng.forward(x.reshape(-1, 784), y, None, nb, stats, train)
    finally:
        fused_cnn._CONV12 = old
    torch.cuda.synchronize()


def _x(seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return torch.randint(0, 256, (B, 1, 28, 28), dtype=torch.uint8, device="cuda", generator=g)


def _decode_pool(val_nchw, am, H):
    """Expand pooled values to the pre-pool map using the kernel's argmax codes."""
    Bn, C, h, w = val_nchw.shape
    out = torch.zeros(Bn, C, H, H, device=val_nchw.device)
    a = am.long()
    alive = a < 4
    dy, dx = (a.clamp(max=3) >> 1), (a.clamp(max=3) & 1)
    py = torch.arange(h, device=a.device).view(1, 1, h, 1).expand_as(a)
    px = torch.arange(w, device=a.device).view(1, 1, 1, w).expand_as(a)
    bi = torch.arange(Bn, device=a.device).view(Bn, 1, 1, 1).expand_as(a)
    ci = torch.arange(C, device=a.device).view(1, C, 1, 1).expand_as(a)
    out[bi[alive], ci[alive], (2 * py + dy)[alive], (2 * px + dx)[alive]] = val_nchw[alive]
    return out


def test_conv1_fwd(eng):
    x = _x(1)
    _forward(eng, x)
    w, b = _p(eng, "conv1.weight"), _p(eng, "conv1.bias")
    conv = F.relu(F.conv2d(x.float() / 255.0, w, b, padding=2))
    ref = F.max_pool2d(conv, 2)  # [B,32,14,14]
    got = eng.p1.view(B, 14, 14, 32).permute(0, 3, 1, 2).float()
    assert _close(got, _bf(ref), rtol=8e-3, atol=1e-6) == 0.0
    # argmax codes point at the maximum of each 2x2 window (or 4 = ReLU-dead)
    am = eng.am1.view(B, 14, 14, 32).permute(0, 3, 1, 2).long()
    alive = am < 4
    a = am.clamp(max=3)
    py = torch.arange(14, device="cuda").view(1, 1, 14, 1)
    px = torch.arange(14, device="cuda").view(1, 1, 1, 14)
    flat = ((2 * py + (a >> 1)) * 28 + 2 * px + (a & 1)).reshape(B, 32, 196)
    picked = conv.reshape(B, 32, 784).gather(2, flat).view(B, 32, 14, 14)
    torch.testing.assert_close(picked[alive], ref[alive], atol=1e-5, rtol=1e-5)
    assert bool(((am == 4) == (ref <= 0)).all())


def test_conv1_shifted_planar_copies(eng):
    x = _x(8)
    _forward(eng, x, train=True)
    p1 = eng.p1.view(B, 14, 14, 32).permute(0, 3, 1, 2)  # [B,32,14,14]
    pad = F.pad(p1.float(), (2, 6, 2, 2))  # [B,32,18,22]: P1pad plus room for the kx shift
    want = torch.stack([pad[..., kx : kx + 16] for kx in range(5)], 1)  # [B,5,32,18,16]
    got = eng.p1s.view(-1, 5, 32, 18, 16)[:B].float()
    assert torch.equal(got, want)


def test_conv2_fwd(eng):
    x = _x(2)
    _forward(eng, x)
    p1 = eng.p1.view(B, 14, 14, 32).permute(0, 3, 1, 2).float()
    w, b = _bf(_p(eng, "conv2.weight")), _p(eng, "conv2.bias")
    ref = F.max_pool2d(F.relu(F.conv2d(p1, w, b, padding=2)), 2).reshape(B, -1)  # [B,3136]
    got = eng.a1.view(-1, 3136)[:B].float()
    assert _close(got, _bf(ref), rtol=1e-2, atol=1e-4) < 1e-3


@pytest.mark.parametrize("train", [True, False])
@pytest.mark.parametrize("nb", [B, 5])
def test_conv12_fwd_bitwise_equals_two_kernels(eng, train, nb):
    """conv1 + conv2 in one launch (P1 window recomputed per pooled-row block in LDS)
    writes exactly what conv1_fwd + conv2_fwd write: P1, AM1, P1s, A1 and AM2 bitwise
    (same fp32 conv1 arithmetic, same MFMA sequence for conv2), full and ragged batches."""
    x = _x(11 + nb).reshape(-1, 784)
    idx = torch.randperm(B, device="cuda")[:nb].contiguous()
    C, M = eng.C, eng.mrows
    bufs = {}
    for fused in (False, True):
        p1 = torch.full((M * 196 * 32,), 7, dtype=torch.bfloat16, device="cuda")
        am1 = torch.full((M * 196 * 32,), 9, dtype=torch.uint8, device="cuda")
        p1s = torch.full((M * 5 * 32 * 18 * 16,), 3, dtype=torch.bfloat16, device="cuda") if train else None
        a1 = torch.zeros(M * 3136, dtype=torch.bfloat16, device="cuda")
        am2 = torch.full((M * 3136,), 9, dtype=torch.uint8, device="cuda")
        if fused:
            C.conv12_fwd(x, idx, eng.params, eng.off, eng.w2r, p1, am1, p1s, a1, am2, nb, M)
        else:
            C.conv1_fwd(x, idx, eng.params, eng.off, p1, am1, p1s, nb)
            C.conv2_fwd(p1, eng.w2r, eng.params, eng.off, a1, am2, nb, M)
        torch.cuda.synchronize()
        bufs[fused] = (p1, am1, p1s, a1, am2)
    for name, u, v in zip(("p1", "am1", "p1s", "a1", "am2"), bufs[False], bufs[True]):
        if u is not None:
            assert torch.equal(u, v), name


@pytest.mark.parametrize("N,K,S", [(2048, 3136, 7), (3136, 2048, 4), (64, 128, 3)])
def test_gemm_skinny(eng, N, K, S):
    g = torch.Generator(device="cuda").manual_seed(N + K)
    A = torch.randn(32, K, device="cuda", generator=g).to(torch.bfloat16)
    Bt = torch.randn(N, K, device="cuda", generator=g).to(torch.bfloat16)
    slabs = torch.zeros(S * 32 * N, device="cuda")
    eng.C.gemm_skinny(A, Bt, slabs, 32, N, K, S)
    got = slabs.view(S, 32, N).sum(0)
    want = A.float() @ Bt.float().t()
    torch.testing.assert_close(got, want, atol=2e-3 * K**0.5, rtol=1e-4)


@pytest.mark.parametrize("w2_bf16", [False, True])
def test_head_and_fc2_wgrad(eng, w2_bf16):
    """Head (FC1 epilogue, FC2, cross-entropy, dH) reading W2 in fp32 or from its bf16
    copy (the reference is then taken on the bf16-rounded W2); then the FC2 gradient."""
    g = torch.Generator(device="cuda").manual_seed(7)
    slabs = torch.randn(eng.S1 * 32 * 2048, device="cuda", generator=g) * 0.05
    labels = torch.randint(0, 10, (B,), device="cuda", generator=g)
    stats = torch.zeros(4, device="cuda")
    w2bf = _p(eng, "l2.weight").to(torch.bfloat16).contiguous() if w2_bf16 else None
    eng.C.head(slabs, eng.S1, 32, eng.params, eng.off, labels, None, B, True, eng.H, eng.dH, eng.dlogits, stats, w2bf)
    torch.cuda.synchronize()
    b1, w2, b2 = _p(eng, "l1.bias"), _p(eng, "l2.weight"), _p(eng, "l2.bias")
    if w2_bf16:
        w2 = _bf(w2)
    h = F.relu(slabs.view(eng.S1, 32, 2048).sum(0)[:B] + b1)
    logits = h @ w2.t() + b2
    loss = F.cross_entropy(logits, labels, reduction="sum")
    dlog = (torch.softmax(logits, 1) - F.one_hot(labels, 10).float()) / B
    dh = (dlog @ w2) * (h > 0)
    assert abs(float(stats[0]) - float(loss)) < 1e-3 * float(loss) + 1e-3
    assert int(stats[1]) == int((logits.argmax(1) == labels).sum())
    torch.testing.assert_close(eng.dlogits.view(-1, 10)[:B], dlog, atol=1e-6, rtol=1e-4)
    torch.testing.assert_close(eng.H.view(-1, 2048)[:B].float(), _bf(h), atol=1e-7, rtol=8e-3)  # <= 1 bf16 ulp
    torch.testing.assert_close(eng.dH.view(-1, 2048)[:B].float(), _bf(dh), atol=1e-7, rtol=8e-3)
    # FC2 gradient (+Adam) from the same H / dlogits
    eng.gdump = torch.zeros_like(eng.params)
    before = eng.params.clone()
    eng.adam_t.fill_(1)
    m_save, v_save = eng.m.clone(), eng.v.clone()
    eng.C.route_fc2(eng.dH, eng.w1_route, eng.am2, 32, B, eng.dc2m, eng.gb, eng.dlogits, eng.H,
                    eng.params, eng.m, eng.v, eng.gdump, eng.off, eng.adam_t, 0, *eng._adam(), row_major=eng.route_rm)
    torch.cuda.synchronize()
    gw = eng.gdump[eng.off[6] : eng.off[6] + 20480].view(10, 2048)
    gb = eng.gdump[eng.off[7] : eng.off[7] + 10]
    torch.testing.assert_close(gw, dlog.t() @ _bf(h), atol=1e-6, rtol=1e-4)
    torch.testing.assert_close(gb, dlog.sum(0), atol=1e-6, rtol=1e-4)
    # first Adam step moves every weight with a non-zero gradient by ~lr
    moved = (eng.params[eng.off[6] : eng.off[6] + 20480] - before[eng.off[6] : eng.off[6] + 20480]).abs()
    assert float(moved.max()) <= 1.0001e-3
    eng.params.copy_(before)
    eng.m.copy_(m_save)
    eng.v.copy_(v_save)
    eng.gdump = None


def test_fc1_wgrad_adam(eng):
    g = torch.Generator(device="cuda").manual_seed(9)
    dh = (torch.randn(32, 2048, device="cuda", generator=g) * 1e-2).to(torch.bfloat16)
    a1 = torch.rand(32, 3136, device="cuda", generator=g).to(torch.bfloat16)
    dht, a1t = dh.t(), a1.t()
    before, m0, v0 = eng.params.clone(), eng.m.clone(), eng.v.clone()
    eng.gdump = torch.zeros_like(eng.params)
    eng.adam_t.fill_(1)
    eng.C.fc1_wgrad_adam(dh, a1, 32, eng.params, eng.m, eng.v, eng.gdump, eng.w1bf, eng.w1tbf, eng.off, eng.adam_t, 0, *eng._adam())
    torch.cuda.synchronize()
    o, ob = eng.off[4], eng.off[5]
    gw = eng.gdump[o : o + 2048 * 3136].view(2048, 3136)
    torch.testing.assert_close(gw, dht.float() @ a1t.float().t(), atol=1e-6, rtol=1e-4)
    torch.testing.assert_close(eng.gdump[ob : ob + 2048], dht.float().sum(1), atol=1e-6, rtol=1e-4)
    # Adam: reference update from the same gradient
    p_ref, m_ref, v_ref = before[o : o + 2048 * 3136].clone(), m0[o : o + 2048 * 3136].clone(), v0[o : o + 2048 * 3136].clone()
    ops.adam_step_reference(p_ref, gw.flatten(), m_ref, v_ref, eng.lr, eng.betas[0], eng.betas[1], eng.eps, eng.wd, 1)
    torch.testing.assert_close(eng.params[o : o + 2048 * 3136], p_ref, atol=1e-6, rtol=1e-5)
    # bf16 shadows are the updated weights, in both layouts
    W = eng.params[o : o + 2048 * 3136].view(2048, 3136)
    assert torch.equal(eng.w1bf.view(2048, 3136), W.to(torch.bfloat16))
    if eng.w1tbf is not None:
        assert torch.equal(eng.w1tbf.view(3136, 2048), W.t().to(torch.bfloat16))
    eng.params.copy_(before)
    eng.m.copy_(m0)
    eng.v.copy_(v0)
    eng.gdump = None
    eng.pack_shadows()


def _route(eng, seed, row_major=None, split=None):
    """Random dH through route_fc2 (dA1 = dH W1, pool2/ReLU backward) into the dC2 map.

    The launch's FC2-Adam blocks update scratch copies, not the engine's weights.
    ``row_major`` picks the kernel reading W1 (LDS transpose reads) or a W1^T
    shadow (built here when the engine keeps none); default: the engine's.
    ``split`` (row-major only) runs the 2-slice split-K variant with its
    in-launch reduction; default: the engine's choice.
    """
    g = torch.Generator(device="cuda").manual_seed(seed)
    dh = (torch.randn(32, 2048, device="cuda", generator=g) * 1e-2).to(torch.bfloat16)
    P, Mm, V = eng.params.clone(), eng.m.clone(), eng.v.clone()
    rm = eng.route_rm if row_major is None else row_major
    w1 = eng.w1bf if rm else eng.w1bf.view(2048, 3136).t().contiguous()
    sp = (eng.route_ws is not None) if split is None else split
    ws = ctr = None
    if rm and sp:
        ws = eng.route_ws if eng.route_ws is not None else torch.zeros(98 * 2 * 32 * 32, device="cuda")
        ctr = eng.route_ctr if eng.route_ctr is not None else torch.zeros(98, dtype=torch.int32, device="cuda")
    eng.C.route_fc2(dh, w1, eng.am2, 32, B, eng.dc2m, eng.gb, eng.dlogits, eng.H,
                    P, Mm, V, None, eng.off, eng.adam_t, 1, *eng._adam(), row_major=rm, ws=ws, ctr=ctr)
    torch.cuda.synchronize()
    return dh


@pytest.mark.parametrize("row_major,split", [(True, True), (True, False), (False, False)])
def test_gemm_da1_route(eng, row_major, split):
    x = _x(6)
    _forward(eng, x)
    dh = _route(eng, 21, row_major, split)
    w1 = _bf(_p(eng, "l1.weight"))
    da1 = dh.float() @ w1  # [32, 3136]
    am2 = eng.am2.view(-1, 3136)[:B]
    alive = am2 < 4
    torch.testing.assert_close(eng.gb.view(-1, 3136)[:B], da1[:B] * alive, atol=1e-5, rtol=1e-3)
    want = _decode_pool(da1[:B].view(B, 64, 7, 7), am2.view(B, 64, 7, 7), 14)
    m = eng.dc2m.view(-1, 64, 14, 16)[:B]
    assert _close(m[..., :14], _bf(want), rtol=8e-3, atol=1e-6) < 1e-4
    assert not bool(m[..., 14:].any())  # row padding stays zero


def test_route_split_k_repeatable(eng):
    """Split-K routing: the tile tickets return to zero after every launch, and the
    slice-order reduction makes repeated launches bitwise identical."""
    x = _x(6)
    _forward(eng, x)
    outs = []
    for _ in range(3):
        _route(eng, 21, True, True)
        outs.append((eng.gb.clone(), eng.dc2m.clone()))
    for gb, dc in outs[1:]:
        assert torch.equal(gb, outs[0][0]) and torch.equal(dc, outs[0][1])
    if eng.route_ctr is not None:
        assert not bool(eng.route_ctr.any())


def test_conv2_bwd(eng):
    """conv2_bwd: conv2 weight gradient (wgrad role) and dP1 -> conv1 weight/bias gradient (dgrad role)."""
    x = _x(3)
    _forward(eng, x, train=True)
    _route(eng, 11)
    eng.C.conv2_bwd(eng.dc2m, eng.p1s, eng.am1, eng.w2q, x.reshape(-1, 784), None, eng.wslab1, eng.wslab2, B)
    torch.cuda.synchronize()
    dc2 = eng.dc2m.view(-1, 64, 14, 16)[:B, :, :, :14].float()
    # wgrad
    p1 = eng.p1.view(B, 14, 14, 32).permute(0, 3, 1, 2).float()
    want_w2 = torch.nn.grad.conv2d_weight(p1, (64, 32, 5, 5), dc2, padding=2)
    ng = eng.C.wgrad_groups(B)
    ws2 = eng.wslab2[: ng * 51200].view(ng, 25, 64, 32).sum(0)  # [tap][oc][ic]
    torch.testing.assert_close(ws2.permute(1, 2, 0).reshape(64, 32, 5, 5), want_w2, atol=1e-6, rtol=2e-3)
    # dgrad + conv1 wgrad
    w2 = _bf(_p(eng, "conv2.weight"))
    dp1 = torch.nn.grad.conv2d_input((B, 32, 14, 14), w2, dc2, padding=2)
    am1 = eng.am1.view(B, 14, 14, 32).permute(0, 3, 1, 2)
    dc1 = _decode_pool(dp1, am1, 28)
    want_w1 = torch.nn.grad.conv2d_weight(x.float() / 255.0, (32, 1, 5, 5), dc1, padding=2)
    ws1 = eng.wslab1[: B * 7 * 832].view(B * 7, 832).sum(0)
    torch.testing.assert_close(ws1[:800].view(32, 1, 5, 5), want_w1, atol=1e-6, rtol=2e-3)
    torch.testing.assert_close(ws1[800:], dc1.sum((0, 2, 3)), atol=1e-6, rtol=1e-3)


@pytest.mark.parametrize("Bp", [7, 1])
def test_conv2_bwd_partial_batch(eng, Bp):
    """Odd / tiny batches: the last wgrad image pair holds one image."""
    x = _x(9)
    _forward(eng, x, True, Bp)  # two-kernel forward: the reference below reads its P1
    g = torch.Generator(device="cuda").manual_seed(5)
    dh = (torch.randn(32, 2048, device="cuda", generator=g) * 1e-2).to(torch.bfloat16)
    dh[Bp:] = 0
    P, Mm, V = eng.params.clone(), eng.m.clone(), eng.v.clone()
    eng.C.route_fc2(dh, eng.w1_route, eng.am2, 32, Bp, eng.dc2m, eng.gb, eng.dlogits, eng.H, P, Mm, V, None, eng.off,
                    eng.adam_t, 1, *eng._adam(), row_major=eng.route_rm, ws=eng.route_ws, ctr=eng.route_ctr)
    eng.C.conv2_bwd(eng.dc2m, eng.p1s, eng.am1, eng.w2q, x.reshape(-1, 784), None, eng.wslab1, eng.wslab2, Bp)
    torch.cuda.synchronize()
    dc2 = eng.dc2m.view(-1, 64, 14, 16)[:Bp, :, :, :14].float()
    p1 = eng.p1.view(-1, 14, 14, 32)[:Bp].permute(0, 3, 1, 2).float()
    want = torch.nn.grad.conv2d_weight(p1, (64, 32, 5, 5), dc2, padding=2)
    ng = eng.C.wgrad_groups(Bp)
    got = eng.wslab2[: ng * 51200].view(ng, 25, 64, 32).sum(0).permute(1, 2, 0).reshape(64, 32, 5, 5)
    torch.testing.assert_close(got, want, atol=1e-6, rtol=2e-3)


def test_conv_adam_and_shadows(eng):
    g = torch.Generator(device="cuda").manual_seed(13)
    ng = eng.C.wgrad_groups(B)
    ws1 = torch.randn(B * 7 * 832, device="cuda", generator=g) * 1e-3
    ws2 = torch.randn(ng * 51200, device="cuda", generator=g) * 1e-3
    gb = torch.randn(B * 3136, device="cuda", generator=g) * 1e-3
    before, m0, v0 = eng.params.clone(), eng.m.clone(), eng.v.clone()
    eng.gdump = torch.zeros_like(eng.params)
    eng.adam_t.fill_(1)
    eng.C.conv_adam(ws1, ws2, gb, B, eng.params, eng.m, eng.v, eng.gdump, eng.w2r, eng.w2q, eng.off, eng.adam_t, 0, *eng._adam())
    torch.cuda.synchronize()
    o = eng.off
    s1 = ws1.view(B * 7, 832).sum(0)
    torch.testing.assert_close(eng.gdump[o[0] : o[0] + 800], s1[:800], atol=1e-7, rtol=1e-5)
    torch.testing.assert_close(eng.gdump[o[1] : o[1] + 32], s1[800:], atol=1e-7, rtol=1e-5)
    w2g = ws2.view(ng, 25, 64, 32).sum(0).permute(1, 2, 0).reshape(-1)
    torch.testing.assert_close(eng.gdump[o[2] : o[2] + 51200], w2g, atol=1e-7, rtol=1e-5)
    torch.testing.assert_close(eng.gdump[o[3] : o[3] + 64], gb.view(B, 64, 49).sum((0, 2)), atol=1e-6, rtol=1e-4)
    p_ref, m_ref, v_ref = before[o[2] : o[2] + 51200].clone(), m0[o[2] : o[2] + 51200].clone(), v0[o[2] : o[2] + 51200].clone()
    # Adam from the kernel's own (checked above) gradient: near-zero sums are
    # order-sensitive and Adam's first step amplifies that to ~lr
    ops.adam_step_reference(p_ref, eng.gdump[o[2] : o[2] + 51200].clone(), m_ref, v_ref, eng.lr, eng.betas[0], eng.betas[1], eng.eps, eng.wd, 1)
    torch.testing.assert_close(eng.params[o[2] : o[2] + 51200], p_ref, atol=1e-6, rtol=1e-5)
    W = eng.params[o[2] : o[2] + 51200].view(64, 32, 25)
    assert torch.equal(eng.w2r.view(64, 25, 32), W.permute(0, 2, 1).to(torch.bfloat16))
    assert torch.equal(eng.w2q.view(32, 25, 64), W.permute(1, 2, 0).to(torch.bfloat16))
    eng.params.copy_(before)
    eng.m.copy_(m0)
    eng.v.copy_(v0)
    eng.gdump = None
    eng.pack_shadows()


def test_bf16_reference_has_similar_gradient_error():
    """Calibrates the end-to-end gradient tolerance: torch's own bf16 autocast vs fp32."""
    torch.manual_seed(0)
    m32 = CNN(seed=2).cuda()
    m16 = CNN(seed=2).cuda()
    x = _x(5).float() / 255.0
    y = torch.randint(0, 10, (B,), device="cuda")
    F.cross_entropy(m32(x), y).backward()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        loss = F.cross_entropy(m16(x), y)
    loss.backward()
    rel = {
        n: float((p16.grad - p32.grad).norm() / p32.grad.norm())
        for (n, p32), (_, p16) in zip(m32.named_parameters(), m16.named_parameters())
    }
    print("torch bf16-autocast vs fp32 gradient rel err:", rel)



def test_w2_bf16_copy_tracks_the_fp32_weight():
    """The head's bf16 FC2 weight is refreshed by every training step's Adam launch and
    by pack_shadows: after steps it equals the fp32 master rounded to bf16."""
    from p2pfl_amd.learning import fused_cnn
    from p2pfl_amd.learning.fused_cnn import FusedCNNEngine

    if not fused_cnn._MERGED_ADAM:
        pytest.skip("the bf16 W2 copy is kept on the merged-Adam path only")
    e = FusedCNNEngine(CNN(seed=5).cuda(), device=torch.device("cuda"))
    o = e.off[6]
    assert torch.equal(e.w2bf, e.params[o : o + 20480].to(torch.bfloat16))
    x = _x(4).reshape(-1, 784)
    y = torch.randint(0, 10, (B,), device="cuda")
    for _ in range(3):
        e.train_step(x, y)
    torch.cuda.synchronize()
    w2 = e.params[o : o + 20480]
    assert torch.equal(e.w2bf, w2.to(torch.bfloat16))


def test_conv2_fwd_eval_sized_launch(eng):
    """The evaluation passes' 128-image launches take the LDS-staged conv2 (B > 64): same
    reference check as test_conv2_fwd, on 100 images."""
    nb, M = 100, 128
    g = torch.Generator(device="cuda").manual_seed(17)
    x = torch.randint(0, 256, (nb, 784), dtype=torch.uint8, device="cuda", generator=g)
    p1 = torch.zeros(M * 196 * 32, dtype=torch.bfloat16, device="cuda")
    am1 = torch.zeros(M * 196 * 32, dtype=torch.uint8, device="cuda")
    a1 = torch.zeros(M * 3136, dtype=torch.bfloat16, device="cuda")
    am2 = torch.zeros(M * 3136, dtype=torch.uint8, device="cuda")
    eng.C.conv1_fwd(x, None, eng.params, eng.off, p1, am1, None, nb)
    eng.C.conv2_fwd(p1, eng.w2r, eng.params, eng.off, a1, am2, nb, M)
    torch.cuda.synchronize()
    p1f = p1.view(M, 14, 14, 32)[:nb].permute(0, 3, 1, 2).float()
    w, b = _bf(_p(eng, "conv2.weight")), _p(eng, "conv2.bias")
    ref = F.max_pool2d(F.relu(F.conv2d(p1f, w, b, padding=2)), 2).reshape(nb, -1)
    assert _close(a1.view(-1, 3136)[:nb].float(), _bf(ref), rtol=1e-2, atol=1e-4) < 1e-3
