"""Implicit-GEMM 2-D convolution on the MFMA core (``csrc/conv.hip``).

:func:`conv2d` runs a ``nn.Conv2d`` (no bias, groups 1) whose activations are
channels-last bf16 and whose weight is a channels-last bf16 view (the
learner's mixed-precision shadow arena, ``arena.py``) on the hand-written
kernels: forward, input gradient and weight gradient are one launch each
(a split-K launch reduces its K-slices itself: ``ops/splitk.py``).  The weight gradient
comes back in the weight's own (O, kh, kw, C) layout, so autograd hands it to
the optimizer without a relayout copy.

Anything the kernels do not take -- CPU tensors, fp32 weights, channel
counts that are not multiples of 64 on the reduction side (the 3-channel
stem), groups, asymmetric stride/padding -- runs ``F.conv2d``.  Where both
can run, the first eager call of each layer shape times native vs MIOpen
and keeps the faster (``ops/autotune.py``; ``P2PFL_NATIVE_CONV=1/0`` forces
one side).  The
reference trains its convolutions through torch.nn.Conv2d
(/root/reference/p2pfl/learning/pytorch/mnist_examples/models/cnn.py:55-62).
"""

from __future__ import annotations

import os
from typing import Optional, Tuple

import torch
import torch.nn.functional as F
from torch import nn

from p2pfl_amd.ops import autotune
from p2pfl_amd.ops.splitk import counters, slab_elems, tiles_of

# counters a test can read to prove the native path ran
STATS = {"native_fwd": 0, "torch_fwd": 0, "gemm_1x1_fwd": 0, "stem_fwd": 0, "native_fwd_bn": 0, "bn_act_conv": 0}
# Training BatchNorm statistics computed by the producing convolution's launch
# (conv_bn_act, csrc/gemm_core.h BnEpi) -- opt-in (P2PFL_CONV_BN_STATS=1).  Off by
# default because it measures slower than the separate statistics + finalize
# launches: per launch the per-tile statistics add ~6.5 us and the cross-workgroup
# reduction (two last-arriver levels, each a ~2-3 us dependent hand-off between
# CUs) ~14.5 us, and its split-K must reduce in the launch (+6-12 us on the
# 16x16 / 8x8 / 4x4 stages), against ~9.6 us for the two separate launches
# (scripts/bn_epi_probe.py; ResNet-18 round 59.9 vs 49.8 ms; profiles/r4_bn_epilogue.md).
_FUSED_BN = os.environ.get("P2PFL_CONV_BN_STATS", "0") == "1"

# env P2PFL_NATIVE_CONV: "library" runs MIOpen for every eager convolution; "native" or "auto"
# (default) run the implicit-GEMM kernels wherever native_ok holds
_POLICY = autotune.policy("P2PFL_NATIVE_CONV")
# csrc/gemm.h variant bits per product (single LDS buffer for the gathers, double buffer for split-K wgrad)
_V_FWD = int(os.environ.get("P2PFL_CONV_VARIANT_FWD", "10"))
_V_DGRAD = int(os.environ.get("P2PFL_CONV_VARIANT_DGRAD", "10"))
_V_WGRAD = int(os.environ.get("P2PFL_CONV_VARIANT_WGRAD", "2"))


def _C():
    from p2pfl_amd.ops import ext

    return ext()


def _sym(v) -> int:
    if isinstance(v, (tuple, list)):
        if len(set(v)) != 1:
            return -1
        return int(v[0])
    return int(v)


def out_hw(h: int, w: int, k: Tuple[int, int], stride: int, pad: int, dil: int) -> Tuple[int, int]:
    return (h + 2 * pad - dil * (k[0] - 1) - 1) // stride + 1, (w + 2 * pad - dil * (k[1] - 1) - 1) // stride + 1


def wgrad_splits(O: int, ncols: int, npix: int) -> int:
    """Split the pixel reduction of a weight gradient until ~2 workgroups per CU."""
    tiles = -(-O // 128) * -(-ncols // 128)
    s = 1
    while tiles * s < 512 and npix // (s * 2) >= 512 and s < 64:
        s *= 2
    return s


def mn_splits(M: int, N: int, K: int, tile: int = 128) -> int:
    """Split-K for a forward / input-gradient product whose output has few tile x tile
    tiles (the 8x8 and 4x4 stages of a CIFAR ResNet): aim at one workgroup per CU, >= 256 deep."""
    tiles = -(-M // tile) * -(-N // tile)
    s = 1
    while tiles * s < 256 and K // (s * 2) >= 256 and s < 16:
        s *= 2
    return s


# Convolutions reduce their split-K slabs with the chip-wide tile_slab_reduce
# launch even at 2-4 slices: measured faster than the in-launch last-arriver
# reduction on every CIFAR ResNet-18 shape (e.g. 128x16x16 forward, 4 slices:
# 19.5 vs 22.7 us; profiles/r3_conv_native.md).  The in-launch path (needed by
# GEMMs with a fused epilogue) stays available: P2PFL_CONV_IN_LAUNCH_SPLITS=4.
_CONV_IN_LAUNCH_MAX_SPLITS = int(os.environ.get("P2PFL_CONV_IN_LAUNCH_SPLITS", "1"))


def _run_split(launch, rows: int, cols: int, s: int, out: torch.Tensor, variant: int = 0,
               in_launch: Optional[bool] = None) -> None:
    """``launch(target, splits, ws, counters)`` producing ``out``: directly, split-K reduced
    in the launch, or split-K into fp32 slabs (fragment-native tiles) reduced by one
    ``tile_slab_reduce`` launch (``variant``: the launch's tile order; ``in_launch``
    None: in the launch up to P2PFL_CONV_IN_LAUNCH_SPLITS slices)."""
    if s == 1:
        launch(out, 1, None, None)
        return
    ws = torch.empty(s * slab_elems(rows, cols), dtype=torch.float32, device=out.device)
    if in_launch if in_launch is not None else s <= _CONV_IN_LAUNCH_MAX_SPLITS:
        launch(out, s, ws, counters(tiles_of(rows, cols, 64 if variant & T64 else 128), out.device))
        return
    launch(ws, s, None, None)
    _C().tile_slab_reduce(ws, s, rows, cols, out.view(rows, cols), variant)


# Per-shape launch configuration.  One fixed (variant, split-K) per direction left
# whole stages on the floor: the CIFAR ResNet's 16x16 / 8x8 stages give 128-256
# output tiles, one workgroup per CU, and the single-LDS-buffer kernel (variant
# bit 3, chosen for occupancy on big grids) then waits a full load latency per
# K-tile (l2 3x3 stride-2 input gradient: 21 us for 8 K-tiles, scripts/conv_one.py
# under rocprofv3).  The first eager call of each (direction, shape) times the
# single-buffer, double-buffer and 4-stage-ring kernels at the default split-K
# and 2x / 4x it (and, for a stride-2 input gradient, the by-phase and the
# all-taps products) and keeps the fastest -- captured step graphs replay it.
# P2PFL_CONV_TUNE=0: the fixed defaults.
_TUNE = os.environ.get("P2PFL_CONV_TUNE", "1") != "0"
_TUNE_VARIANTS = (10, 2, 4096 | 2)
# csrc/gemm.h kConvT64: 64 x 64 output tiles (gemm_core.h Tile64).  The 16x16 / 8x8 / 4x4
# stages get 4x the tiles of a 128 x 128 grid -- the chip fills without split-K slabs and
# their reduce launch -- and 64-channel products stop running half of every MFMA on
# zero columns.  Offered beside the 128 x 128 kernels (single / double buffer, 4-stage
# ring) with its own split-K options; P2PFL_CONV_T64=0 withdraws it.
T64 = 1 << 14
_T64 = os.environ.get("P2PFL_CONV_T64", "1") != "0"
_TUNE_VARIANTS_T64 = (T64 | 10, T64 | 2, T64 | 4096 | 2)
# the 64 x 64 tiles' split-K also reduced in the launch (P2PFL_CONV_T64_IL=0: slabs + reduce only)
_T64_IL = os.environ.get("P2PFL_CONV_T64_IL", "1") != "0"


def _split_options(base: int, K: int, min_k: int = 128) -> Tuple[int, ...]:
    """The default split-K and up to two doublings that keep >= min_k of K per slice."""
    out = [base]
    while len(out) < 3 and K // (out[-1] * 2) >= min_k and out[-1] < 64:
        out.append(out[-1] * 2)
    return tuple(out)


def _configs(prefix: str, make, default_variant: int, splits) -> dict:
    """Candidates ``{name: run(dst)}`` of one path: every tuned variant x split-K (untuned:
    the default variant).  Split-K reduces through slabs + tile_slab_reduce: the in-launch
    reduction (``_run_split(..., in_launch=True)``) was also offered per shape and never won
    a ResNet-18 product (``profiles/r5_conv_bench.md``)."""
    pre = f"{prefix}_" if prefix else ""
    return {f"{pre}v{v}_s{sp}": make(v, sp) for v in (_TUNE_VARIANTS if _TUNE else (default_variant,)) for sp in splits}


def _configs_t64(prefix: str, make, splits) -> dict:
    """The 64 x 64-tile candidates of one path (tuned runs only; P2PFL_CONV_T64=0: none):
    each variant x split-K through slabs + tile_slab_reduce, and (suffix ``_il``) the
    split-K reduced in the launch by the last-arriving slice (no reduce launch)."""
    if not (_TUNE and _T64):
        return {}
    pre = f"{prefix}_" if prefix else ""
    out = {f"{pre}v{v}_s{sp}": make(v, sp) for v in _TUNE_VARIANTS_T64 for sp in splits}
    if _T64_IL:
        out.update({f"{pre}v{v}_s{sp}_il": make(v, sp, True) for v in _TUNE_VARIANTS_T64 for sp in splits if sp > 1})
    return out


def _pick(key, cands, default: str, out: torch.Tensor) -> None:
    """Run ``cands[name](out)`` for the measured-fastest name of ``key`` (``default``
    untuned, or unseen inside a capture); candidates are timed into a scratch output."""
    if not _TUNE or len(cands) == 1:
        cands[default](out)
        return
    scratch = []

    def timed(f):
        def run():
            if not scratch:
                scratch.append(torch.empty_like(out))
            f(scratch[0])
        return run

    name = autotune.choose(key, [(n, timed(f)) for n, f in cands.items()], default=default)
    cands[name](out)


# stride-2 input gradients by output phase (env P2PFL_CONV_S2_PHASES=0: the all-taps gather)
_S2_PHASES = os.environ.get("P2PFL_CONV_S2_PHASES", "1") != "0"


def s2_phases_ok(stride: int, dil: int, dx_shape, k: Tuple[int, int] = (3, 3)) -> bool:
    """Shapes csrc/conv.hip conv_dgrad_s2 takes: stride 2, no dilation, even H and W,
    and whole 128-row tiles per phase (N H W / 4 % 128 == 0).  Not offered for 1x1
    kernels: one phase of the output, but the extra interleave launch made it slower
    than the gather (l3 shortcut 8.6 -> 14.4 us; the models run 1x1 convolutions as
    GEMMs anyway, conv1x1_gemm)."""
    N, H, W = dx_shape[0], dx_shape[1], dx_shape[2]
    return (_S2_PHASES and stride == 2 and dil == 1 and k[0] * k[1] > 1 and H % 2 == 0 and W % 2 == 0
            and (N * H * W // 4) % 128 == 0)


def dgrad_into(dy4: torch.Tensor, w4: torch.Tensor, stride: int, pad: int, dil: int, dx4: torch.Tensor) -> None:
    """dX [N, H, W, C] bf16 <- conv input gradient of dY [N, OH, OW, O] and W [O, kh, kw, C]
    (NHWC views).  Stride 2: by output phase (csrc/conv.hip ConvDgradS2A: ~4x fewer
    K-tiles for 3x3 than gathering all taps) then phase_interleave, or the all-taps
    gather (ConvDgradA), whichever configuration measured faster (:func:`_pick`)."""
    C = _C()
    shape = list(dx4.shape)
    O, kh, kw = w4.shape[0], w4.shape[1], w4.shape[2]
    rows = shape[0] * shape[1] * shape[2]
    K = kh * kw * O

    def gather(v, sp, il=None):
        return lambda dst: _run_split(
            lambda o, s, ws, cnt: C.conv_dgrad(dy4, w4, stride, pad, dil, o, shape, s, v, ws, cnt),
            rows, shape[3], sp, dst, v, il)

    def phases(v, sp, il=None):
        def run(dst):
            ph = torch.empty((rows, shape[3]), dtype=torch.bfloat16, device=dx4.device)
            _run_split(lambda o, s, ws, cnt: C.conv_dgrad_s2(dy4, w4, pad, o, shape, s, v, ws, cnt),
                       rows, shape[3], sp, ph, v, il)
            C.phase_interleave(ph, dst, pad, kh, kw)
        return run

    base = mn_splits(rows, shape[3], K)
    cands = _configs("gather", gather, _V_DGRAD, _split_options(base, K))
    cands.update(_configs_t64("gather", gather, _split_options(mn_splits(rows, shape[3], K, 64), K)))
    default = f"gather_v{_V_DGRAD}_s{base}"
    if s2_phases_ok(stride, dil, shape, (kh, kw)):
        kq = ((kh + 1) // 2) * ((kw + 1) // 2) * O  # K of one phase
        pbase = mn_splits(rows, shape[3], kq)
        cands.update(_configs("phase", phases, _V_DGRAD, _split_options(pbase, kq)))
        cands.update(_configs_t64("phase", phases, _split_options(mn_splits(rows, shape[3], kq, 64), kq)))
        default = f"phase_v{_V_DGRAD}_s{pbase}"
        cands.setdefault(default, phases(_V_DGRAD, pbase))
    cands.setdefault(default, gather(_V_DGRAD, base))
    _pick(("conv_dgrad", tuple(shape), O, kh, kw, stride, pad, dil), cands, default, dx4)


def fwd_into(x4: torch.Tensor, w4: torch.Tensor, stride: int, pad: int, dil: int, y4: torch.Tensor) -> None:
    """Y [N, OH, OW, O] bf16 <- conv of X [N, H, W, C] and W [O, kh, kw, C] (NHWC views),
    in the measured-fastest (variant, split-K) of the shape (:func:`_pick`)."""
    C = _C()
    N, OH, OW, O = y4.shape
    kh, kw, Cin = w4.shape[1], w4.shape[2], w4.shape[3]
    rows, K = N * OH * OW, kh * kw * Cin

    def one(v, sp, il=None):
        return lambda dst: _run_split(lambda o, s, ws, cnt: C.conv_fwd(x4, w4, stride, pad, dil, o, s, v, ws, cnt),
                                      rows, O, sp, dst, v, il)

    base = mn_splits(rows, O, K)
    cands = _configs("", one, _V_FWD, _split_options(base, K))
    cands.update(_configs_t64("", one, _split_options(mn_splits(rows, O, K, 64), K)))
    _pick(("conv_fwd", tuple(x4.shape), O, kh, kw, stride, pad, dil), cands, f"v{_V_FWD}_s{base}", y4)


def wgrad_into(dy4: torch.Tensor, x4: torch.Tensor, stride: int, pad: int, dil: int, dw4: torch.Tensor) -> None:
    """dW [O, kh, kw, C] <- conv weight gradient (NHWC views), in the measured-fastest
    (variant, split-K) of the shape (:func:`_pick`; splits: the default, half and double)."""
    C = _C()
    O, kh, kw, Cin = dw4.shape
    npix = dy4.shape[0] * dy4.shape[1] * dy4.shape[2]
    ncols = kh * kw * Cin

    def one(v, sp, il=None):
        return lambda dst: _run_split(
            lambda o, s, ws, cnt: C.conv_wgrad(dy4, x4, kh, kw, stride, pad, dil, o, s, v, ws, cnt), O, ncols, sp, dst, v,
            il)

    base = wgrad_splits(O, ncols, npix)
    splits = sorted({max(1, base // 2), base} | ({base * 2} if npix // (base * 2) >= 256 else set()))
    cands = _configs("", one, _V_WGRAD, splits)
    cands.update(_configs_t64("", one, splits))
    default = f"v{_V_WGRAD}_s{base}"
    if default not in cands:
        cands[default] = one(_V_WGRAD, base)
    _pick(("conv_wgrad", tuple(x4.shape), O, kh, kw, stride, pad, dil), cands, default, dw4)


def native_ok(x: torch.Tensor, conv: nn.Conv2d) -> bool:
    from p2pfl_amd.ops import _gpu

    if not _gpu(x) or x.dim() != 4:
        return False
    w = conv.weight
    if w.dtype != torch.bfloat16 or conv.bias is not None or conv.groups != 1 or conv.padding_mode != "zeros":
        return False
    if isinstance(conv.padding, str):
        return False
    stride, pad, dil = _sym(conv.stride), _sym(conv.padding), _sym(conv.dilation)
    if stride not in (1, 2) or pad < 0 or dil < 1:
        return False
    O, C = w.shape[0], w.shape[1]
    if C % 64 or O % 64:
        return False
    if not w.permute(0, 2, 3, 1).is_contiguous() or w.data_ptr() % 16:
        return False
    return x.shape[1] == C and x.is_contiguous(memory_format=torch.channels_last)


class _Conv2dNHWC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, stride, pad, dil):
        if x.dtype != torch.bfloat16:
            x = x.to(torch.bfloat16)
        x4 = x.permute(0, 2, 3, 1)
        if not x4.is_contiguous() or x4.data_ptr() % 16:
            x4 = x4.contiguous()
        w4 = w.permute(0, 2, 3, 1)
        N, H, W_, C = x4.shape
        O, kh, kw = w4.shape[0], w4.shape[1], w4.shape[2]
        OH, OW = out_hw(H, W_, (kh, kw), stride, pad, dil)
        y4 = torch.empty((N, OH, OW, O), dtype=torch.bfloat16, device=x.device)
        fwd_into(x4, w4, stride, pad, dil, y4)
        ctx.save_for_backward(x4, w)
        ctx.cfg = (stride, pad, dil)
        return y4.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, dy):
        x4, w = ctx.saved_tensors
        stride, pad, dil = ctx.cfg
        if dy.dtype != torch.bfloat16:
            dy = dy.to(torch.bfloat16)
        dy4 = dy.permute(0, 2, 3, 1)
        if not dy4.is_contiguous() or dy4.data_ptr() % 16:
            dy4 = dy4.contiguous()
        w4 = w.permute(0, 2, 3, 1)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx4 = torch.empty(x4.shape, dtype=torch.bfloat16, device=x4.device)
            dgrad_into(dy4, w4, stride, pad, dil, dx4)
            dx = dx4.permute(0, 3, 1, 2)
        if ctx.needs_input_grad[1]:
            dw4 = torch.empty(w4.shape, dtype=w.dtype, device=w.device)
            wgrad_into(dy4, x4, stride, pad, dil, dw4)
            dw = dw4.permute(0, 3, 1, 2)
        return dx, dw, None, None, None


def _nhwc_bf16(t: torch.Tensor) -> torch.Tensor:
    """[N, C, H, W] channels-last (bf16) -> its contiguous, 16-byte aligned NHWC storage view."""
    if t.dtype != torch.bfloat16:
        t = t.to(torch.bfloat16)
    t4 = t.permute(0, 2, 3, 1)
    if not t4.is_contiguous() or t4.data_ptr() % 16:
        t4 = t4.contiguous()
    return t4


def _fwd_bn_launch(x4, w, stride, pad, dil, bn_w, bn_b, rm, rv, nbt, eps, momentum):
    """One conv_fwd_bn launch: (y4 NHWC bf16, mean, rstd, coef) -- the forward product
    plus the training BatchNorm statistics of its output (split-K reduced in the launch)."""
    from p2pfl_amd.ops import splitk

    w4 = w.permute(0, 2, 3, 1)
    N, H, W_, C = x4.shape
    O, kh, kw = w4.shape[0], w4.shape[1], w4.shape[2]
    OH, OW = out_hw(H, W_, (kh, kw), stride, pad, dil)
    y4 = torch.empty((N, OH, OW, O), dtype=torch.bfloat16, device=x4.device)
    rows = N * OH * OW
    s = mn_splits(rows, O, kh * kw * C)
    ws = cnt = None
    if s > 1:  # in-launch reduction: the statistics epilogue sees whole tiles
        ws = torch.empty(s * slab_elems(rows, O), dtype=torch.float32, device=x4.device)
        cnt = counters(tiles_of(rows, O), x4.device)
    tiles_m, tiles_n = -(-rows // 128), -(-O // 128)
    groups = -(-tiles_m // 16)
    part = torch.empty((tiles_m + groups) * 2 * O, dtype=torch.float32, device=x4.device)
    bcnt = splitk.counters(tiles_n * (groups + 1), x4.device)
    f32 = dict(dtype=torch.float32, device=x4.device)
    mean, rstd, coef = torch.empty(O, **f32), torch.empty(O, **f32), torch.empty(3 * O, **f32)
    _C().conv_fwd_bn(x4, w4, stride, pad, dil, y4, s, _V_FWD, ws, cnt, part, bcnt, bn_w, bn_b, rm, rv, nbt,
                     mean, rstd, coef, float(eps), float(momentum))
    return y4, mean, rstd, coef


def _wgrad_launch(dy4, x4, w, stride, pad, dil):
    dw4 = torch.empty(w.permute(0, 2, 3, 1).shape, dtype=w.dtype, device=w.device)
    wgrad_into(dy4, x4, stride, pad, dil, dw4)
    return dw4.permute(0, 3, 1, 2)


class _Conv2dNHWCBN(torch.autograd.Function):
    """:class:`_Conv2dNHWC` whose launch also computes the training BatchNorm
    statistics of its bf16 output (``gemm_core.h`` BnEpi: per-tile column moments,
    reduced by the last-arriving tiles, finalized in the same launch) -- the BN
    statistics and finalize passes of ``csrc/batchnorm.hip`` disappear.  Returns
    (y, mean, rstd, coef); the three statistics are not differentiable."""

    @staticmethod
    def forward(ctx, x, w, stride, pad, dil, bn_w, bn_b, rm, rv, nbt, eps, momentum):
        x4 = _nhwc_bf16(x)
        y4, mean, rstd, coef = _fwd_bn_launch(x4, w, stride, pad, dil, bn_w, bn_b, rm, rv, nbt, eps, momentum)
        ctx.save_for_backward(x4, w)
        ctx.cfg = (stride, pad, dil)
        ctx.mark_non_differentiable(mean, rstd, coef)
        ctx.set_materialize_grads(False)  # no zero-filled gradients for the three statistics
        return y4.permute(0, 3, 1, 2), mean, rstd, coef

    @staticmethod
    def backward(ctx, dy, _dmean, _drstd, _dcoef):
        dx, dw, _, _, _ = _Conv2dNHWC.backward(ctx, dy)
        return dx, dw, None, None, None, None, None, None, None, None, None, None


class _BNActConvBN(torch.autograd.Function):
    """``y2 = conv(act(bn1(y1)))`` + bn2's training statistics, where bn1's batch
    statistics (mean1, rstd1, coef1) came from the launch that produced y1.

    Forward: bn1's apply pass, then one ``conv_fwd_bn`` launch.  Backward: ONE
    input-gradient launch also reduces bn1's backward statistics (``conv_dgrad_bn``:
    sum dz', sum dz' (y1 - mean1), finalized into dgamma1, dbeta1 and the apply
    coefficients), then bn1's backward apply pass gives dy1 -- bn1's separate
    backward statistics and finalize passes disappear -- and the weight gradient.
    """

    @staticmethod
    def forward(ctx, y1, g1, b1, mean1, rstd1, coef1, relu1, w, stride, pad, dil, bn_w, bn_b, rm, rv, nbt, eps, momentum):
        from p2pfl_amd.ops.batchnorm import _bx

        y14 = _nhwc_bf16(y1)
        C = y14.shape[3]
        z4 = _bx().apply_train(y14.reshape(-1, C), None, coef1, bool(relu1)).view(y14.shape)
        y24, mean, rstd, coef = _fwd_bn_launch(z4, w, stride, pad, dil, bn_w, bn_b, rm, rv, nbt, eps, momentum)
        ctx.save_for_backward(y14, z4, w, g1, mean1, rstd1)
        ctx.cfg = (stride, pad, dil, bool(relu1))
        ctx.mark_non_differentiable(mean, rstd, coef)
        ctx.set_materialize_grads(False)
        return y24.permute(0, 3, 1, 2), mean, rstd, coef

    @staticmethod
    def backward(ctx, dy, _dmean, _drstd, _dcoef):
        from p2pfl_amd.ops import splitk
        from p2pfl_amd.ops.batchnorm import _bx

        y14, z4, w, g1, mean1, rstd1 = ctx.saved_tensors
        stride, pad, dil, relu1 = ctx.cfg
        dy4 = _nhwc_bf16(dy)
        w4 = w.permute(0, 2, 3, 1)
        shape = list(y14.shape)
        O, kh, kw = w4.shape[0], w4.shape[1], w4.shape[2]
        C = shape[3]
        rows = shape[0] * shape[1] * shape[2]
        dx4 = torch.empty(y14.shape, dtype=torch.bfloat16, device=dy4.device)
        s = mn_splits(rows, C, kh * kw * O)
        ws = cnt = None
        if s > 1:
            ws = torch.empty(s * slab_elems(rows, C), dtype=torch.float32, device=dy4.device)
            cnt = counters(tiles_of(rows, C), dy4.device)
        tiles_m, tiles_n = -(-rows // 128), -(-C // 128)
        groups = -(-tiles_m // 16)
        part = torch.empty((tiles_m + groups) * 2 * C, dtype=torch.float32, device=dy4.device)
        bcnt = splitk.counters(tiles_n * (groups + 1), dy4.device)
        f32 = dict(dtype=torch.float32, device=dy4.device)
        dg, db, coefb = torch.empty(C, **f32), torch.empty(C, **f32), torch.empty(3 * C, **f32)
        _C().conv_dgrad_bn(dy4, w4, stride, pad, dil, dx4, shape, s, _V_DGRAD, ws, cnt, part, bcnt, g1, y14,
                           z4 if relu1 else None, mean1, rstd1, dg, db, coefb)
        dy1 = _bx().apply_bwd(dx4.view(rows, C), z4.view(rows, C) if relu1 else None, y14.view(rows, C), mean1, coefb)
        dy1 = dy1.view(y14.shape).permute(0, 3, 1, 2)
        dw = _wgrad_launch(dy4, z4, w, stride, pad, dil) if ctx.needs_input_grad[7] else None
        return (dy1, dg.to(g1.dtype), db.to(g1.dtype), None, None, None, None, dw) + (None,) * 10


def conv_bn_stats(x: torch.Tensor, conv: nn.Conv2d, bn: nn.BatchNorm2d):
    """``(y, mean, rstd, coef)``: ``conv(x)`` on the native kernels with bn's training
    statistics computed by the same launch, or None when that path does not apply."""
    from p2pfl_amd.ops import batchnorm as bnops

    capturing = x.is_cuda and torch.cuda.is_current_stream_capturing()
    if not (_FUSED_BN and bnops.fused_stats_ok(bn) and native_ok(x, conv) and (capturing or _POLICY != "library")):
        return None
    track = bn.track_running_stats
    rm = bn.running_mean if track else None
    rv = bn.running_var if track else None
    nbt = bn.num_batches_tracked if track and bn.num_batches_tracked is not None else None
    STATS["native_fwd_bn"] += 1
    return _Conv2dNHWCBN.apply(x, conv.weight, _sym(conv.stride), _sym(conv.padding), _sym(conv.dilation), bn.weight,
                               bn.bias, rm, rv, nbt, bn.eps, bn.momentum)


def bn_act_conv_bn_stats(st, bn1: nn.BatchNorm2d, relu1: bool, conv: nn.Conv2d, bn: nn.BatchNorm2d):
    """Given ``st = (y1, mean1, rstd1, coef1)`` from :func:`conv_bn_stats` (or this
    function), ``conv(act(bn1(y1)))`` with bn's statistics from the same launch
    (:class:`_BNActConvBN`), or None when that path does not apply."""
    from p2pfl_amd.ops import batchnorm as bnops

    y1, mean1, rstd1, coef1 = st
    capturing = y1.is_cuda and torch.cuda.is_current_stream_capturing()
    if not (_FUSED_BN and bnops.fused_stats_ok(bn) and native_ok(y1, conv) and (capturing or _POLICY != "library")
            and conv.weight.shape[0] % 64 == 0):
        return None
    track = bn.track_running_stats
    rm = bn.running_mean if track else None
    rv = bn.running_var if track else None
    nbt = bn.num_batches_tracked if track and bn.num_batches_tracked is not None else None
    STATS["native_fwd_bn"] += 1
    STATS["bn_act_conv"] += 1
    return _BNActConvBN.apply(y1, bn1.weight, bn1.bias, mean1, rstd1, coef1, bool(relu1), conv.weight, _sym(conv.stride),
                              _sym(conv.padding), _sym(conv.dilation), bn.weight, bn.bias, rm, rv, nbt, bn.eps, bn.momentum)


def conv_bn_act(x: torch.Tensor, conv: nn.Conv2d, bn: nn.BatchNorm2d, residual=None, relu: bool = True, fork: bool = False):
    """``act(bn(conv(x)) [+ residual])``.  In training, on the native implicit-GEMM
    kernels, the convolution's launch computes the batch statistics (and updates the
    running ones): only the BN apply pass remains a separate launch.  Anything else
    composes :func:`conv2d` and :func:`~p2pfl_amd.ops.batchnorm.batch_norm_act`.
    ``fork``: return the pair of :func:`~p2pfl_amd.ops.batchnorm.batch_norm_act`."""
    from p2pfl_amd.ops import batchnorm as bnops

    if residual is None or residual.is_contiguous(memory_format=torch.channels_last):
        st = conv_bn_stats(x, conv, bn)
        if st is not None:
            if residual is not None and residual.shape != st[0].shape:
                raise ValueError("conv_bn_act: residual shape mismatch")
            return bnops.batch_norm_apply(st[0], bn, st[1], st[2], st[3], residual, relu, fork)
    return bnops.batch_norm_act(conv2d(x, conv), bn, residual=residual, relu=relu, fork=fork)


# 1x1 convolutions (ResNet-50 bottlenecks and downsample shortcuts) run as the
# GEMM they are: NHWC pixels x C times W^T, through ops.gemm.linear (native MFMA
# GEMM or hipBLASLt, measured per shape; all memory from PyTorch's allocator).
# MIOpen solves them with GEMM-based solvers whose library-internal workspace
# is not graph-safe: replayed in a captured step graph they corrupted the
# weight gradients whenever PyTorch's allocator had to map new segments
# (profiles/r3_nan_root_cause.md).  P2PFL_CONV1X1_GEMM=0 restores conv2d.
_ONE_BY_ONE_GEMM = os.environ.get("P2PFL_CONV1X1_GEMM", "1") != "0"
# Where a 1x1 convolution runs, eager and captured alike (P2PFL_CONV1X1_MODE):
#   "conv"   (default) the implicit-GEMM conv kernels in both, tuned per shape by the eager
#            step (64 x 64 tiles included), so the captured step replays measured choices;
#   "gemm"   ops.gemm.linear in both (the GEMM is native-only, so graph-safe; under
#            P2PFL_NATIVE_GEMM=library a capture takes the conv kernels);
#   "legacy" round 5: GEMM eagerly, conv kernels inside a capture -- where no eager call
#            had timed them, so every captured 1x1 ran the untuned default configuration.
# Measured (MI355X, bench.py --steps 8, scripts/ab_conv1x1.sh): ResNet-50 conv 103.6 /
# gemm 121.5 / legacy 108.8 ms per round; ResNet-18 conv 38.9 / gemm 40.7 ms.
_1X1_MODE = os.environ.get("P2PFL_CONV1X1_MODE", "conv")


def _is_1x1(x: torch.Tensor, conv: nn.Conv2d) -> bool:
    from p2pfl_amd.ops import _gpu

    return (_ONE_BY_ONE_GEMM and _gpu(x) and x.dim() == 4 and tuple(conv.kernel_size) == (1, 1) and conv.groups == 1
            and _sym(conv.padding) == 0 and _sym(conv.dilation) == 1 and _sym(conv.stride) in (1, 2)
            and conv.padding_mode == "zeros" and conv.weight.shape[0] % 8 == 0 and conv.weight.shape[1] % 8 == 0)


def conv1x1_gemm(x: torch.Tensor, conv: nn.Conv2d) -> torch.Tensor:
    """``conv(x)`` for a 1x1 convolution as a GEMM over channels-last pixels (stride 2: every
    other row / column first).  Returns a channels-last NCHW tensor; autograd flows through
    the view ops and :func:`p2pfl_amd.ops.gemm.linear`."""
    from p2pfl_amd.ops.gemm import linear

    s = _sym(conv.stride)
    x4 = x.permute(0, 2, 3, 1)
    if s == 2:
        x4 = x4[:, ::2, ::2, :]
    N, H, W_, C = x4.shape
    O = conv.weight.shape[0]
    y2 = linear(x4.reshape(N * H * W_, C), conv.weight.reshape(O, C), conv.bias)
    STATS["gemm_1x1_fwd"] += 1
    return y2.view(N, H, W_, O).permute(0, 3, 1, 2)


def conv2d(x: torch.Tensor, conv: nn.Conv2d) -> torch.Tensor:
    """``conv(x)`` on the implicit-GEMM kernels whenever they take the shape (:func:`native_ok`),
    eager or captured alike -- MIOpen only under ``P2PFL_NATIVE_CONV=library`` or for shapes the
    kernels refuse; 1x1 convolutions as GEMMs (:func:`conv1x1_gemm`)."""
    # Inside a HIP-graph capture the implicit-GEMM kernels run whatever the
    # eager timing preferred: MIOpen convolutions replayed from captured step
    # graphs corrupted weights as soon as several learners' graphs and eager
    # steps shared the device (profiles/r3_nan_root_cause.md); eager steps may
    # no longer take MIOpen either (the short last batch of an epoch used to
    # autotune against it).  This holds under every policy, "library" included,
    # and for 1x1 convolutions too (no hipBLASLt GEMM inside a graph).
    capturing = x.is_cuda and torch.cuda.is_current_stream_capturing()
    if _1X1_MODE == "gemm" and _is_1x1(x, conv):
        import importlib

        if not capturing or importlib.import_module("p2pfl_amd.ops.gemm")._POLICY != "library":
            return conv1x1_gemm(x, conv)
    if capturing and native_ok(x, conv):
        STATS["native_fwd"] += 1
        return _Conv2dNHWC.apply(x, conv.weight, _sym(conv.stride), _sym(conv.padding), _sym(conv.dilation))
    if _1X1_MODE == "legacy" and _is_1x1(x, conv):
        return conv1x1_gemm(x, conv)
    if x.shape[1] < 8 and stem_ok(x, conv) and _POLICY != "library":
        return stem_conv2d(x, conv)
    if native_ok(x, conv) and _POLICY != "library":
        STATS["native_fwd"] += 1
        return _Conv2dNHWC.apply(x, conv.weight, _sym(conv.stride), _sym(conv.padding), _sym(conv.dilation))
    STATS["torch_fwd"] += 1
    if x.is_cuda:
        import importlib

        if importlib.import_module("p2pfl_amd.ops.gemm").STRICT:
            raise RuntimeError(f"native convolution refused {tuple(x.shape)} x {tuple(conv.weight.shape)} "
                               f"stride {conv.stride} pad {conv.padding} (P2PFL_STRICT_NATIVE=1)")
    return conv(x)


# ---- small-C direct convolution: the 3-channel stem (csrc/stem.hip) -------------------
def stem_ok(x: torch.Tensor, conv: nn.Conv2d) -> bool:
    """The stem kernels take this convolution: few input channels (kh*kw*C <= 160),
    O in {32, 64}, bf16 channels-last weight, symmetric stride/padding, no bias, and an
    input that needs no gradient (it is data)."""
    from p2pfl_amd.ops import _gpu

    if not _gpu(x) or x.dim() != 4 or x.dtype not in (torch.float32, torch.bfloat16, torch.uint8):
        return False
    if torch.is_grad_enabled() and x.requires_grad:
        return False
    w = conv.weight
    if w.dtype != torch.bfloat16 or conv.bias is not None or conv.groups != 1 or conv.padding_mode != "zeros":
        return False
    if isinstance(conv.padding, str) or _sym(conv.dilation) != 1:
        return False
    stride, pad = _sym(conv.stride), _sym(conv.padding)
    O, C, kh, kw = w.shape
    if stride < 1 or stride > 4 or pad < 0 or pad > 8 or C != x.shape[1] or O not in (32, 64):
        return False
    if kh * kw * C > 160 or kh * kw * C * O * 4 > 40 * 1024:
        return False
    return w.permute(0, 2, 3, 1).is_contiguous() and w.data_ptr() % 16 == 0


class _StemConv(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, stride, pad, xscale):
        w4 = w.permute(0, 2, 3, 1)
        N, _, H, W_ = x.shape
        O, kh, kw = w4.shape[0], w4.shape[1], w4.shape[2]
        OH, OW = out_hw(H, W_, (kh, kw), stride, pad, 1)
        y4 = torch.empty((N, OH, OW, O), dtype=torch.bfloat16, device=x.device)
        _C().stem_fwd(x, w4, stride, pad, xscale, y4)
        ctx.save_for_backward(x, w)
        ctx.cfg = (stride, pad, xscale)
        return y4.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        stride, pad, xscale = ctx.cfg
        dw = None
        if ctx.needs_input_grad[1]:
            if dy.dtype != torch.bfloat16:
                dy = dy.to(torch.bfloat16)
            dy4 = dy.permute(0, 2, 3, 1)
            if not dy4.is_contiguous() or dy4.data_ptr() % 16:
                dy4 = dy4.contiguous()
            w4 = w.permute(0, 2, 3, 1)
            C = _C()
            parts = C.stem_wgrad_parts(dy4.shape[0], dy4.shape[1], dy4.shape[2])
            part = torch.empty(parts * w4.numel(), dtype=torch.float32, device=w.device)
            dw4 = torch.empty(w4.shape, dtype=w.dtype, device=w.device)
            C.stem_wgrad(dy4, x, w4, stride, pad, xscale, part, dw4)
            dw = dw4.permute(0, 3, 1, 2)
        return None, dw, None, None, None


def stem_conv2d(x: torch.Tensor, conv: nn.Conv2d, xscale: float = 1.0) -> torch.Tensor:
    """``conv(x * xscale)`` on the small-C direct kernels (:func:`stem_ok` must hold); x in
    any layout / fp32, bf16 or uint8; returns a channels-last bf16 NCHW tensor."""
    STATS["stem_fwd"] += 1
    return _StemConv.apply(x, conv.weight, _sym(conv.stride), _sym(conv.padding), float(xscale))


def conv2d_reference(x: torch.Tensor, w: torch.Tensor, stride: int, pad: int, dil: int) -> torch.Tensor:
    """fp32 definition used by the numerics tests."""
    return F.conv2d(x.float(), w.float(), None, stride, pad, dil)
