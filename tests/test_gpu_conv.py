"""Implicit-GEMM convolutions (csrc/conv.hip) vs an fp32 PyTorch reference on the same bf16 operands."""

from __future__ import annotations

import pytest
import torch
import torch.nn.functional as F
from torch import nn

from p2pfl_amd import ops
from p2pfl_amd.ops import conv as conv_ops

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _require_ext(monkeypatch):
    ops.ext()
    # these tests exercise the hand-written kernels: no per-shape library choice
    monkeypatch.setattr(conv_ops, "_POLICY", "native")
    monkeypatch.setattr(conv_ops, "_ONE_BY_ONE_GEMM", False)  # 1x1 shapes here test the implicit-GEMM kernels


def _operands(N, C, H, W, O, k, seed, integer=False):
    g = torch.Generator(device="cuda").manual_seed(seed)
    if integer:  # exact in bf16 and fp32: any mis-addressed tap shows as an exact mismatch
        x = torch.randint(-2, 3, (N, C, H, W), device="cuda", generator=g).float()
        w = torch.randint(-2, 3, (O, C, k, k), device="cuda", generator=g).float()
    else:
        x = torch.randn(N, C, H, W, device="cuda", generator=g)
        w = torch.randn(O, C, k, k, device="cuda", generator=g) / (C * k * k) ** 0.5
    xb = x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    wb = w.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    return xb, wb


CASES = [
    # N, C, H, W, O, k, stride, pad, dil
    (2, 64, 8, 8, 64, 3, 1, 1, 1),
    (2, 64, 8, 8, 128, 3, 2, 1, 1),
    (3, 128, 7, 5, 64, 3, 1, 1, 1),
    (2, 64, 9, 9, 128, 1, 2, 0, 1),
    (2, 128, 6, 6, 64, 1, 1, 0, 1),
    (1, 64, 10, 10, 64, 3, 1, 2, 2),
    (4, 64, 32, 32, 64, 3, 1, 1, 1),
    (2, 256, 4, 4, 512, 3, 2, 1, 1),
]


def _ref(x, w, s, p, d):
    return F.conv2d(x.float(), w.float(), None, s, p, d)


@pytest.mark.parametrize("N,C,H,W,O,k,s,p,d", CASES)
def test_conv_fwd_exact_integers(N, C, H, W, O, k, s, p, d):
    x, w = _operands(N, C, H, W, O, k, seed=N + C + H + O, integer=True)
    y4 = torch.empty((N,) + conv_ops.out_hw(H, W, (k, k), s, p, d) + (O,), dtype=torch.bfloat16, device="cuda")
    ops.ext().conv_fwd(x.permute(0, 2, 3, 1), w.permute(0, 2, 3, 1), s, p, d, y4, 1)
    ref = _ref(x, w, s, p, d)
    # integer sums up to |k*k*C*4| <= 256 per term class: exact in fp32, and bf16 output holds them when |y| <= 256
    torch.testing.assert_close(y4.permute(0, 3, 1, 2).float(), ref.to(torch.bfloat16).float(), atol=0, rtol=0)


@pytest.mark.parametrize("N,C,H,W,O,k,s,p,d", CASES)
def test_conv_autograd_vs_fp32(N, C, H, W, O, k, s, p, d):
    x, w = _operands(N, C, H, W, O, k, seed=7 * N + C + W + k)
    conv = nn.Conv2d(C, O, k, s, p, d, bias=False).cuda()
    conv.weight.data = w  # bf16 channels-last view, as the mixed-precision arena provides
    xg = x.clone().requires_grad_()
    before = conv_ops.STATS["native_fwd"]
    y = ops.conv2d(xg, conv)
    assert conv_ops.STATS["native_fwd"] == before + 1, "native path not taken"
    g = torch.randn(y.shape, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y.backward(g)
    xr = x.float().requires_grad_()
    wr = w.float().requires_grad_()
    yr = _ref(xr, wr, s, p, d)
    yr.backward(g.float())
    torch.testing.assert_close(y.float(), yr, atol=3e-2, rtol=2e-2)
    torch.testing.assert_close(xg.grad.float(), xr.grad, atol=3e-2, rtol=2e-2)
    scale = wr.grad.abs().max().item()
    torch.testing.assert_close(conv.weight.grad.float(), wr.grad, atol=1e-2 * scale, rtol=2e-2)
    # gradient keeps the weight's channels-last layout (no relayout copy for the optimizer)
    assert conv.weight.grad.permute(0, 2, 3, 1).is_contiguous()


@pytest.mark.parametrize("variant", [10, 4096 | 10])
@pytest.mark.parametrize("splits", [2, 16])
def test_conv_fwd_dgrad_split_k(splits, variant):
    """Raw split-K slabs reduced by tile_slab_reduce with the launch's own variant --
    also the 4-stage-ring conv (bit 12), whose slabs are 128 x 128 tiles like every
    conv kernel's (bit 12 once meant 256 x 256 slabs to the reducer: wrong sums)."""
    N, C, H, W, O, k = 2, 128, 4, 4, 256, 3
    x, w = _operands(N, C, H, W, O, k, seed=splits, integer=True)
    from p2pfl_amd.ops.splitk import slab_elems

    C_ = ops.ext()
    x4, w4 = x.permute(0, 2, 3, 1), w.permute(0, 2, 3, 1)
    rows = N * H * W
    # raw fragment-native slabs (no counters), summed by tile_slab_reduce with the launch's variant
    slabs = torch.empty(splits * slab_elems(rows, O), device="cuda")
    C_.conv_fwd(x4, w4, 1, 1, 1, slabs, splits, variant)
    y = torch.empty(rows, O, device="cuda")
    C_.tile_slab_reduce(slabs, splits, rows, O, y, variant)
    ref = _ref(x, w, 1, 1, 1)
    torch.testing.assert_close(y.view(N, H, W, O).permute(0, 3, 1, 2), ref, atol=0, rtol=0)
    dy = torch.randint(-2, 3, (N, O, H, W), device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    slabs = torch.empty(splits * slab_elems(rows, C), device="cuda")
    C_.conv_dgrad(dy.permute(0, 2, 3, 1), w4, 1, 1, 1, slabs, [N, H, W, C], splits, variant)
    dx = torch.empty(rows, C, device="cuda")
    C_.tile_slab_reduce(slabs, splits, rows, C, dx, variant)
    xr = x.float().requires_grad_()
    _ref(xr, w, 1, 1, 1).backward(dy.float())
    torch.testing.assert_close(dx.view(N, H, W, C).permute(0, 3, 1, 2), xr.grad, atol=0, rtol=0)


@pytest.mark.parametrize("splits", [2, 8, 32])
def test_conv_split_k_in_launch_reduction(splits):
    """Split-K reduced by the last-arriving slice: equals the slab sum, and the counters end at zero."""
    from p2pfl_amd.ops.splitk import slab_elems, tiles_of

    N, C, H, W, O, k = 4, 128, 8, 8, 256, 3
    x, w = _operands(N, C, H, W, O, k, seed=3 * splits, integer=True)
    x4, w4 = x.permute(0, 2, 3, 1), w.permute(0, 2, 3, 1)
    rows = N * H * W
    cnt = torch.zeros(tiles_of(rows, O), dtype=torch.int32, device="cuda")
    ws = torch.empty(splits * slab_elems(rows, max(O, C)), device="cuda")
    y4 = torch.empty(N, H, W, O, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):  # counters are reusable launch after launch
        ops.ext().conv_fwd(x4, w4, 1, 1, 1, y4, splits, 10, ws, cnt)
        ref = _ref(x, w, 1, 1, 1)
        torch.testing.assert_close(y4.permute(0, 3, 1, 2).float(), ref.to(torch.bfloat16).float(), atol=0, rtol=0)
        assert int(cnt.abs().sum()) == 0
    dy = torch.randint(-2, 3, (N, O, H, W), device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dx4 = torch.empty(N, H, W, C, device="cuda", dtype=torch.bfloat16)
    cnt = torch.zeros(tiles_of(rows, C), dtype=torch.int32, device="cuda")
    ops.ext().conv_dgrad(dy.permute(0, 2, 3, 1), w4, 1, 1, 1, dx4, [N, H, W, C], splits, 10, ws, cnt)
    xr = x.float().requires_grad_()
    wr = w.float().requires_grad_()
    _ref(xr, wr, 1, 1, 1).backward(dy.float())
    torch.testing.assert_close(dx4.permute(0, 3, 1, 2).float(), xr.grad.to(torch.bfloat16).float(), atol=0, rtol=0)
    dw4 = torch.empty(O, k, k, C, device="cuda", dtype=torch.float32)
    cnt = torch.zeros(tiles_of(O, k * k * C), dtype=torch.int32, device="cuda")
    ws = torch.empty(splits * slab_elems(O, k * k * C), device="cuda")
    ops.ext().conv_wgrad(dy.permute(0, 2, 3, 1), x4, k, k, 1, 1, 1, dw4, splits, 2, ws, cnt)
    torch.testing.assert_close(dw4, wr.grad.permute(0, 2, 3, 1), atol=0, rtol=0)
    assert int(cnt.abs().sum()) == 0


@pytest.mark.parametrize("N,C,H,W,O,k,s,p,d", CASES)
@pytest.mark.parametrize("variant", [conv_ops.T64 | 10, conv_ops.T64 | 2, conv_ops.T64 | 4096 | 2])
@pytest.mark.parametrize("splits", [1, 3])
def test_conv_t64_tiles_exact(N, C, H, W, O, k, s, p, d, variant, splits):
    """64 x 64 output tiles (csrc/conv.hip conv64_kernel, variant bit 14) in all three
    pipelines: forward, input and weight gradient equal the fp32 products exactly on
    integer operands -- plain stores, and split-K slabs of the 64 x 64 geometry summed by
    tile_slab_reduce with the same variant (ragged M / N tails included)."""
    from p2pfl_amd.ops.splitk import slab_elems

    x, w = _operands(N, C, H, W, O, k, seed=N + C + H + O + variant % 7, integer=True)
    C_ = ops.ext()
    x4, w4 = x.permute(0, 2, 3, 1), w.permute(0, 2, 3, 1)
    OH, OW = conv_ops.out_hw(H, W, (k, k), s, p, d)
    dy = torch.randint(-2, 3, (N, O, OH, OW), device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dy4 = dy.permute(0, 2, 3, 1)
    xr, wr = x.float().requires_grad_(), w.float().requires_grad_()
    yr = _ref(xr, wr, s, p, d)
    yr.backward(dy.float())

    def run(launch, rows, cols, out_bf16):
        if splits == 1:
            out = torch.empty(rows, cols, device="cuda", dtype=torch.bfloat16 if out_bf16 else torch.float32)
            launch(out, 1)
            return out.float()
        slabs = torch.empty(splits * slab_elems(rows, cols), device="cuda")
        launch(slabs, splits)
        out = torch.empty(rows, cols, device="cuda")
        C_.tile_slab_reduce(slabs, splits, rows, cols, out, variant)
        return out

    y = run(lambda o, sp: C_.conv_fwd(x4, w4, s, p, d, o.view(N, OH, OW, O) if sp == 1 else o, sp, variant),
            N * OH * OW, O, True)
    ref_y = yr.detach().permute(0, 2, 3, 1).reshape(-1, O)
    torch.testing.assert_close(y, ref_y.to(torch.bfloat16).float() if splits == 1 else ref_y, atol=0, rtol=0)
    dx = run(lambda o, sp: C_.conv_dgrad(dy4, w4, s, p, d, o.view(N, H, W, C) if sp == 1 else o, [N, H, W, C], sp, variant),
             N * H * W, C, True)
    ref_dx = xr.grad.permute(0, 2, 3, 1).reshape(-1, C)
    torch.testing.assert_close(dx, ref_dx.to(torch.bfloat16).float() if splits == 1 else ref_dx, atol=0, rtol=0)
    dw = run(lambda o, sp: C_.conv_wgrad(dy4, x4, k, k, s, p, d, o.view(O, k, k, C) if sp == 1 else o, sp, variant),
             O, k * k * C, False)
    torch.testing.assert_close(dw, wr.grad.permute(0, 2, 3, 1).reshape(O, -1), atol=0, rtol=0)


@pytest.mark.parametrize("splits", [2, 5])
def test_conv_t64_in_launch_split_k_exact(splits):
    """64 x 64 tiles with the split-K reduced in the launch (last-arriving slice, one
    counter per 64 x 64 tile): exact on integer operands for all three products, and
    the counters are back at zero afterwards."""
    from p2pfl_amd.ops.splitk import slab_elems, tiles_of

    N, C, H, W, O, k = 4, 128, 8, 8, 256, 3
    x, w = _operands(N, C, H, W, O, k, seed=9 * splits, integer=True)
    x4, w4 = x.permute(0, 2, 3, 1), w.permute(0, 2, 3, 1)
    rows, v = N * H * W, conv_ops.T64 | 2
    C_ = ops.ext()
    dy = torch.randint(-2, 3, (N, O, H, W), device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    xr, wr = x.float().requires_grad_(), w.float().requires_grad_()
    yr = _ref(xr, wr, 1, 1, 1)
    yr.backward(dy.float())
    for _ in range(2):  # counters reusable launch after launch
        cnt = torch.zeros(tiles_of(rows, O, 64), dtype=torch.int32, device="cuda")
        ws = torch.empty(splits * slab_elems(rows, max(O, C)), device="cuda")
        y4 = torch.empty(N, H, W, O, device="cuda", dtype=torch.bfloat16)
        C_.conv_fwd(x4, w4, 1, 1, 1, y4, splits, v, ws, cnt)
        torch.testing.assert_close(y4.permute(0, 3, 1, 2).float(), yr.detach().to(torch.bfloat16).float(), atol=0, rtol=0)
        assert int(cnt.abs().sum()) == 0
        cnt = torch.zeros(tiles_of(rows, C, 64), dtype=torch.int32, device="cuda")
        dx4 = torch.empty(N, H, W, C, device="cuda", dtype=torch.bfloat16)
        C_.conv_dgrad(dy.permute(0, 2, 3, 1), w4, 1, 1, 1, dx4, [N, H, W, C], splits, v, ws, cnt)
        torch.testing.assert_close(dx4.permute(0, 3, 1, 2).float(), xr.grad.to(torch.bfloat16).float(), atol=0, rtol=0)
        assert int(cnt.abs().sum()) == 0
        cnt = torch.zeros(tiles_of(O, k * k * C, 64), dtype=torch.int32, device="cuda")
        wsw = torch.empty(splits * slab_elems(O, k * k * C), device="cuda")
        dw4 = torch.empty(O, k, k, C, device="cuda", dtype=torch.float32)
        C_.conv_wgrad(dy.permute(0, 2, 3, 1), x4, k, k, 1, 1, 1, dw4, splits, v, wsw, cnt)
        torch.testing.assert_close(dw4, wr.grad.permute(0, 2, 3, 1), atol=0, rtol=0)
        assert int(cnt.abs().sum()) == 0


S2_CASES = [
    # N, C, H, W, O, k, pad: shapes the by-phase stride-2 input gradient takes (N H W / 4 % 128 == 0)
    (8, 64, 16, 16, 128, 3, 1),
    (8, 128, 16, 16, 256, 1, 0),
    (2, 64, 32, 32, 64, 3, 0),
    (32, 64, 8, 8, 128, 5, 2),
]


@pytest.mark.parametrize("N,C,H,W,O,k,p", S2_CASES)
@pytest.mark.parametrize("mode", ["plain", "slabs", "in_launch"])
def test_conv_dgrad_stride2_by_phase_exact(N, C, H, W, O, k, p, mode):
    """conv_dgrad_s2 + phase_interleave equals the fp32 input gradient exactly on integer
    operands: each phase's taps addressed right, tap-less phases (1x1) zero."""
    from p2pfl_amd.ops.splitk import slab_elems, tiles_of

    x, w = _operands(N, C, H, W, O, k, seed=N + H + k, integer=True)
    OH, OW = conv_ops.out_hw(H, W, (k, k), 2, p, 1)
    dy = torch.randint(-2, 3, (N, O, OH, OW), device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    C_ = ops.ext()
    dy4, w4 = dy.permute(0, 2, 3, 1), w.permute(0, 2, 3, 1)
    rows = N * H * W // (4 if k == 1 else 1)
    ph = torch.empty(rows, C, device="cuda", dtype=torch.bfloat16)
    if mode == "plain":
        C_.conv_dgrad_s2(dy4, w4, p, ph, [N, H, W, C])
    elif mode == "slabs":
        slabs = torch.empty(4 * slab_elems(rows, C), device="cuda")
        C_.conv_dgrad_s2(dy4, w4, p, slabs, [N, H, W, C], 4, 10)
        acc = torch.empty(rows, C, device="cuda")
        C_.tile_slab_reduce(slabs, 4, rows, C, acc, 10)
        ph.copy_(acc)
    else:
        ws = torch.empty(8 * slab_elems(rows, C), device="cuda")
        cnt = torch.zeros(tiles_of(rows, C), dtype=torch.int32, device="cuda")
        C_.conv_dgrad_s2(dy4, w4, p, ph, [N, H, W, C], 8, 10, ws, cnt)
        assert int(cnt.abs().sum()) == 0
    dx4 = torch.full((N, H, W, C), float("nan"), device="cuda", dtype=torch.bfloat16)
    C_.phase_interleave(ph, dx4, p, k, k)
    xr = x.float().requires_grad_()
    _ref(xr, w.float(), 2, p, 1).backward(dy.float())
    torch.testing.assert_close(dx4.permute(0, 3, 1, 2).float(), xr.grad.to(torch.bfloat16).float(), atol=0, rtol=0)


def test_stride2_autograd_takes_phase_path(monkeypatch):
    """The conv autograd's stride-2 input gradient runs by phase (and the all-taps gather
    when switched off) with the same result."""
    N, C, H, W, O, k = 8, 64, 16, 16, 128, 3
    x, w = _operands(N, C, H, W, O, k, seed=11)
    assert conv_ops.s2_phases_ok(2, 1, [N, H, W, C])
    assert not conv_ops.s2_phases_ok(2, 1, [N, H, W, C], (1, 1))
    conv = nn.Conv2d(C, O, k, 2, 1, bias=False).cuda()
    conv.weight.data = w
    grads = []
    for on, tune in ((True, False), (False, False), (True, True)):
        monkeypatch.setattr(conv_ops, "_S2_PHASES", on)
        monkeypatch.setattr(conv_ops, "_TUNE", tune)  # untuned: the default path of each setting
        xg = x.clone().requires_grad_()
        y = ops.conv2d(xg, conv)
        torch.manual_seed(0)
        y.backward(torch.randn(y.shape, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last))
        grads.append(xg.grad.float())
    torch.testing.assert_close(grads[0], grads[1], atol=2e-2, rtol=1e-2)
    torch.testing.assert_close(grads[2], grads[1], atol=2e-2, rtol=1e-2)
    key = ("conv_dgrad", (N, H, W, C), O, k, k, 2, 1, 1)
    assert key in conv_ops.autotune.choices(), "tuned run did not time the stride-2 input gradient"


def test_tuned_configs_all_agree(monkeypatch):
    """Every (variant, split-K) candidate the per-shape tuning may pick gives the same
    exact result on integer operands (forward, input and weight gradient)."""
    N, C, H, W, O, k = 4, 128, 8, 8, 256, 3
    x, w = _operands(N, C, H, W, O, k, seed=5, integer=True)
    dy = torch.randint(-2, 3, (N, O, H, W), device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x4, w4, dy4 = x.permute(0, 2, 3, 1), w.permute(0, 2, 3, 1), dy.permute(0, 2, 3, 1)
    seen = {}

    def grab(key, cands, default, out):
        for name, f in cands.items():
            dst = torch.full_like(out, float("nan"))
            f(dst)
            seen.setdefault(key[0], []).append((name, dst))
        cands[default](out)

    monkeypatch.setattr(conv_ops, "_pick", grab)
    monkeypatch.setattr(conv_ops, "_TUNE", True)
    conv_ops.fwd_into(x4, w4, 1, 1, 1, torch.empty(N, H, W, O, device="cuda", dtype=torch.bfloat16))
    conv_ops.dgrad_into(dy4, w4, 1, 1, 1, torch.empty(N, H, W, C, device="cuda", dtype=torch.bfloat16))
    conv_ops.wgrad_into(dy4, x4, 1, 1, 1, torch.empty(O, k, k, C, device="cuda", dtype=torch.float32))
    xr, wr = x.float().requires_grad_(), w.float().requires_grad_()
    y = _ref(xr, wr, 1, 1, 1)
    y.backward(dy.float())
    refs = {"conv_fwd": y.detach().permute(0, 2, 3, 1).to(torch.bfloat16).float(),
            "conv_dgrad": xr.grad.permute(0, 2, 3, 1).to(torch.bfloat16).float(),
            "conv_wgrad": wr.grad.permute(0, 2, 3, 1)}
    for kind, outs in seen.items():
        assert len(outs) >= 3, kind
        for name, dst in outs:
            torch.testing.assert_close(dst.float(), refs[kind], atol=0, rtol=0, msg=f"{kind} {name}")


@pytest.mark.parametrize("splits", [1, 2, 8, 64])
def test_conv_wgrad_split_k(splits):
    N, C, H, W, O, k = 8, 64, 16, 16, 64, 3
    x, w = _operands(N, C, H, W, O, k, seed=splits)
    dy = torch.randn(N, O, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    from p2pfl_amd.ops.splitk import slab_elems

    n = O * k * k * C
    out = torch.empty((splits * slab_elems(O, k * k * C),) if splits > 1 else (O, k, k, C), dtype=torch.float32, device="cuda")
    ops.ext().conv_wgrad(dy.permute(0, 2, 3, 1), x.permute(0, 2, 3, 1), k, k, 1, 1, 1, out, splits)
    if splits > 1:
        dw = torch.empty(O, k * k * C, device="cuda")
        ops.ext().tile_slab_reduce(out, splits, O, k * k * C, dw, 2)
    else:
        dw = out.view(-1)
    xr = x.float().requires_grad_()
    wr = w.float().requires_grad_()
    _ref(xr, wr, 1, 1, 1).backward(dy.float())
    torch.testing.assert_close(dw.view(O, k, k, C), wr.grad.permute(0, 2, 3, 1), atol=5e-3 * wr.grad.abs().max().item(), rtol=1e-3)


def test_slab_sum():
    slabs = torch.randn(5, 4096, device="cuda")
    out = torch.empty(4096, device="cuda", dtype=torch.bfloat16)
    ops.ext().slab_sum(slabs, out)
    torch.testing.assert_close(out.float(), slabs.sum(0).to(torch.bfloat16).float(), atol=1e-2, rtol=1e-2)


def test_conv_rejects_bad_shapes():
    x = torch.zeros(1, 8, 8, 48, device="cuda", dtype=torch.bfloat16)  # C % 64 != 0
    w = torch.zeros(64, 3, 3, 48, device="cuda", dtype=torch.bfloat16)
    y = torch.empty(1, 8, 8, 64, device="cuda", dtype=torch.bfloat16)
    with pytest.raises(RuntimeError):
        ops.ext().conv_fwd(x, w, 1, 1, 1, y, 1)


def test_resnet18_block_runs_native_convs():
    """A ResNet-18 train step through the learner's mixed-precision arena takes the native conv path."""
    from p2pfl_amd.learning.arena import ModuleArena
    from p2pfl_amd.models.resnet import ResNet18

    torch.manual_seed(0)
    model = ResNet18(num_classes=10).cuda()
    arena = ModuleArena(model, device=torch.device("cuda"), compute_dtype=torch.bfloat16,
                        channels_last_names=model.channels_last_parameter_names())
    x = torch.randint(0, 255, (8, 3, 32, 32), device="cuda", dtype=torch.uint8)
    before = dict(conv_ops.STATS)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        loss = model(x).float().logsumexp(1).mean()
    loss.backward()
    native = sum(conv_ops.STATS[k] - before[k] for k in ("native_fwd", "native_fwd_bn"))
    assert native >= 19, conv_ops.STATS  # every block / shortcut convolution (with the BN statistics epilogue)
    assert conv_ops.STATS["stem_fwd"] - before["stem_fwd"] == 1  # the 3-channel stem, on its direct kernel
    assert conv_ops.STATS["torch_fwd"] - before["torch_fwd"] == 0  # nothing left on MIOpen
    assert torch.isfinite(loss)
    assert arena.shadow is not None
    for name, p in model.named_parameters():
        if p.dim() == 4:
            assert p.grad is not None and torch.isfinite(p.grad).all(), name


def test_auto_policy_runs_native_eagerly(monkeypatch):
    """Policy "auto": eager convolutions run the implicit-GEMM kernels (no MIOpen timing race)."""
    monkeypatch.setattr(conv_ops, "_POLICY", "auto")
    x, w = _operands(2, 64, 8, 8, 64, 3, seed=11)
    conv = nn.Conv2d(64, 64, 3, 1, 1, bias=False).cuda()
    conv.weight.data = w
    before = dict(conv_ops.STATS)
    xg = x.clone().requires_grad_()
    y = ops.conv2d(xg, conv)
    y.float().sum().backward()
    assert conv_ops.STATS["native_fwd"] == before["native_fwd"] + 1
    assert conv_ops.STATS["torch_fwd"] == before["torch_fwd"]
    torch.testing.assert_close(y.float(), _ref(x, w, 1, 1, 1), atol=3e-2, rtol=2e-2)


def test_resnet_fit_with_ragged_last_batch_never_runs_miopen(monkeypatch):
    """A whole fit() -- graph-replayed full batches plus the eager short last batch and the
    validation pass -- runs no MIOpen convolution."""
    from p2pfl_amd.data import Cifar10FederatedDM
    from p2pfl_amd.learning.torch_learner import TorchLearner
    from p2pfl_amd.models.resnet import ResNet18

    monkeypatch.setattr(conv_ops, "_POLICY", "auto")
    data = Cifar10FederatedDM(sub_id=0, number_sub=250, batch_size=32)  # 200 samples: 6 x 32 + 8 train
    assert len(data.train_dataloader().dataset) % 32 != 0
    ln = TorchLearner(ResNet18(seed=0, lr_rate=0.01), data, "p", 1, device=torch.device("cuda", 0))
    before = dict(conv_ops.STATS)
    ln.fit()
    torch.cuda.synchronize()
    assert conv_ops.STATS["torch_fwd"] == before["torch_fwd"]
    assert conv_ops.STATS["native_fwd"] > before["native_fwd"]


# ---- small-C direct convolution (3-channel stem, csrc/stem.hip) -------------------------
STEM_CASES = [
    # N, C, H, W, O, k, stride, pad, x layout
    (4, 3, 32, 32, 64, 3, 1, 1, "nchw"),
    (3, 3, 17, 13, 64, 3, 1, 1, "cl"),
    (2, 3, 40, 40, 64, 7, 2, 3, "nchw"),
    (5, 1, 28, 28, 32, 5, 1, 2, "nchw"),
    (2, 4, 9, 11, 32, 3, 2, 0, "cl"),
]


@pytest.mark.parametrize("N,C,H,W,O,k,s,p,layout", STEM_CASES)
@pytest.mark.parametrize("xdtype", [torch.float32, torch.uint8])
def test_stem_conv_fwd_wgrad_vs_fp32(N, C, H, W, O, k, s, p, layout, xdtype):
    """Forward and weight gradient of the direct small-C kernels against fp32 PyTorch on
    the same bf16-rounded operands (input read in its own layout / dtype, 1/255 folded)."""
    g = torch.Generator(device="cuda").manual_seed(N * 100 + k)
    if xdtype == torch.uint8:
        x = torch.randint(0, 256, (N, C, H, W), device="cuda", generator=g, dtype=torch.uint8)
        scale = 1.0 / 255.0
        xref = (x.float() * scale).to(torch.bfloat16).float()
    else:
        x = torch.randn(N, C, H, W, device="cuda", generator=g)
        scale = 1.0
        xref = x.to(torch.bfloat16).float()
    if layout == "cl":
        x = x.contiguous(memory_format=torch.channels_last)
    conv = nn.Conv2d(C, O, k, s, p, bias=False).cuda()
    with torch.no_grad():
        conv.weight.copy_(torch.randn(O, C, k, k, device="cuda", generator=g) / (C * k * k) ** 0.5)
    conv.weight.data = conv.weight.data.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    assert conv_ops.stem_ok(x, conv)
    y = conv_ops.stem_conv2d(x, conv, scale)
    wr = conv.weight.detach().float().requires_grad_()
    yr = F.conv2d(xref, wr, None, s, p)
    assert y.shape == yr.shape and y.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(y.float(), yr, atol=2e-2, rtol=1e-2)
    dy = torch.randn(yr.shape, device="cuda", generator=g).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y.backward(dy)
    yr.backward(dy.float())
    scale_g = wr.grad.abs().max().item()
    torch.testing.assert_close(conv.weight.grad.float(), wr.grad, atol=1e-2 * scale_g, rtol=1e-2)
    assert conv.weight.grad.is_contiguous(memory_format=torch.channels_last)


def test_stem_wgrad_is_deterministic():
    x = torch.rand(8, 3, 32, 32, device="cuda")
    conv = nn.Conv2d(3, 64, 3, 1, 1, bias=False).cuda()
    conv.weight.data = conv.weight.data.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dy = torch.randn(8, 64, 32, 32, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    grads = []
    for _ in range(3):
        conv.weight.grad = None
        conv_ops.stem_conv2d(x, conv).backward(dy)
        grads.append(conv.weight.grad.clone())
    assert all(torch.equal(grads[0], g) for g in grads[1:])


def test_resnet_stem_runs_native(monkeypatch):
    """ResNet's forward sends the 3-channel stem to the direct kernels (no F.conv2d)."""
    from p2pfl_amd.models.resnet import ResNet18

    m = ResNet18().cuda()
    for mod in m.modules():
        if isinstance(mod, nn.Conv2d):
            mod.weight.data = mod.weight.data.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    calls = []
    monkeypatch.setattr(F, "conv2d", lambda *a, **k: calls.append(a) or torch.zeros(()))
    before = conv_ops.STATS["stem_fwd"]
    x = torch.randint(0, 256, (2, 3, 32, 32), dtype=torch.uint8, device="cuda")
    m.eval()
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        y = m(x)
    assert conv_ops.STATS["stem_fwd"] == before + 1 and not calls and y.shape == (2, 10)
