"""Linear layers on the hand-written MFMA GEMM (``csrc/gemm.hip``).

:func:`gemm` exposes the kernel: ``C = A . B^T`` over bf16 operands with fp32
accumulation, each operand given in its natural memory layout (k-major or
m/n-major, so nothing is transposed in memory), an epilogue with bias, GELU
(+ pre-activation) and residual add, and split-K into fp32 slabs reduced by
the FedAvg weighted-sum kernel (fp32 accumulation, bf16 out).

:func:`linear` / :func:`linear_gelu` are ``nn.Linear`` (and ``gelu(nn.Linear)``)
with all three products -- forward, input gradient, weight gradient -- on
that kernel; the bias gradient is the column-sum kernel.  Reference shapes:
``/root/reference/p2pfl/learning/pytorch/mnist_examples/models/mlp.py:53-69``
and the ViT-B/16 of BASELINE config 4.
"""

from __future__ import annotations

import os

from typing import Optional, Tuple

import torch
import torch.nn.functional as F

from p2pfl_amd.ops import autotune
from p2pfl_amd.ops.splitk import IN_LAUNCH_MAX_SPLITS, counters, slab_elems, tiles_of


def _C():
    from p2pfl_amd.ops import ext

    return ext()


def gemm_reference(a, b, a_kmajor=True, b_kmajor=True, bias=None, gelu=False, residual=None):
    A = a.float() if a_kmajor else a.float().t()
    B = b.float() if b_kmajor else b.float().t()
    c = A @ B.t()
    if bias is not None:
        c = c + bias.float()
    z = c
    if gelu:
        c = F.gelu(c)
    if residual is not None:
        c = c + residual.float()
    return c, z


# Upper bound of the weight-gradient split-K factor (P2PFL_GEMM_MAX_SPLITS).  64: the
# ResNet-50 1x1 weight gradients (K = 32768 pixels, 2-8 tiles) ran at 16 slices on 32
# workgroups; 64 measured 124.0 / 126.3 vs 128.3 / 128.1 ms per round (scripts/r3_gpu34.sh).
_MAX_SPLITS = int(os.environ.get("P2PFL_GEMM_MAX_SPLITS", "64"))


def splits_for(M: int, N: int, K: int) -> int:
    """Split-K factor so that a small M x N grid still covers the 256 CUs."""
    tiles = -(-M // 128) * -(-N // 128)
    s = 1
    while tiles * s < 256 and K // (s * 2) >= 512 and s < _MAX_SPLITS:
        s *= 2
    return s


def supported(M: int, N: int, K: int, a_kmajor: bool, b_kmajor: bool) -> bool:
    """Shapes the kernel takes (checked again, loudly, by the native binding)."""
    if N % 8 or M < 1 or K < 8:
        return False
    if (a_kmajor or b_kmajor) and K % 8:
        return False
    return a_kmajor or M % 8 == 0


# Products the MFMA kernels refuse (N % 8, K % 8 on a k-major operand, ...) fall back
# to torch; every fallback is counted here, and P2PFL_STRICT_NATIVE=1 turns it into an
# error (tests/test_gpu_native_coverage.py runs whole ResNet / ViT fits that way).
STATS = {"native": 0, "torch": 0}
STRICT = os.environ.get("P2PFL_STRICT_NATIVE", "0") == "1"


def torch_fallback(what: str) -> None:
    """Record (or, strict, refuse) a GPU product that leaves the hand-written kernels."""
    STATS["torch"] += 1
    if STRICT:
        raise RuntimeError(f"native GEMM path refused {what} (P2PFL_STRICT_NATIVE=1)")


def _product(a, b, a_kmajor, b_kmajor, dtype, splits=1):
    """One Linear product on the MFMA kernel, or torch for shapes it does not take."""
    M = a.shape[0] if a_kmajor else a.shape[1]
    N = b.shape[0] if b_kmajor else b.shape[1]
    K = a.shape[1] if a_kmajor else a.shape[0]
    if supported(M, N, K, a_kmajor, b_kmajor):
        STATS["native"] += 1
        return gemm(a, b, a_kmajor, b_kmajor, out_dtype=dtype, splits=splits)[0]
    torch_fallback(f"M={M} N={N} K={K} a_kmajor={a_kmajor} b_kmajor={b_kmajor}")
    A = a if a_kmajor else a.t()
    B = b if b_kmajor else b.t()
    return (A @ B.t()).to(dtype)


# Kernel schedule per product (csrc/gemm.h variant bits; measured on the ViT
# shapes, profiles/r2_gemm_variants.md): forward / input-gradient products run
# the single-LDS-buffer schedule (4 workgroups per CU hide the DMA latency)
# with A-panel tile order; the split-K weight gradient keeps the double buffer.
_VARIANT_ENV = os.environ.get("P2PFL_GEMM_VARIANT")


PP = 2048  # variant bit 11: the ping-pong 256 x 256 pipeline (csrc/gemm_pp.hip)
PP_M16 = 1 << 16  # with PP: the same pipeline on v_mfma_f32_16x16x32_bf16
PP_SK = 1 << 17  # with PP: stream-K schedule, ``splits`` = grid size (csrc/gemm_pp.hip)
PP_N128 = 1 << 21  # with PP: the 256 x 128 output tile (150 whole tiles for the N = 768 products)
PP_ROWSPLIT = 1 << 22  # with PP: rows split into one full wave of 256 x 256 tiles + a 256 x 128 tail launch
# split-K reduced in the launch (last-arriving slice per tile) at any slice count, not only up to
# IN_LAUNCH_MAX_SPLITS: a configuration bit of this module, never passed to the kernels
GEMM_IL = 1 << 23
SK_SLAB = 256 * 256  # fp32 elements of one stream-K partial tile (two per workgroup)


def sk_iters(M: int, N: int, K: int) -> int:
    """K-tile iterations a stream-K launch divides among its workgroups."""
    return -(-M // 256) * -(-N // 256) * -(-K // 64)


def pp_eligible(M: int, N: int, K: int, a_kmajor: bool, b_kmajor: bool) -> bool:
    """Products the ping-pong kernel takes and wins on (profiles/r3_gemm_pingpong.md):
    at least ~150 tiles of 256 x 256 (below that one partial wave of big tiles
    loses to the 128 x 128 tile), and no K tail in a k-major operand (k-major
    tails are not caught by its buffer range check)."""
    tiles = -(-M // 256) * -(-N // 256)
    return tiles >= 150 and (K % 64 == 0 or not (a_kmajor or b_kmajor))


def pp_eligible_any(M: int, N: int, K: int, a_kmajor: bool, b_kmajor: bool) -> bool:
    """Products the ping-pong kernel takes at all (csrc/gemm_pp.hip gemm_pp_supported)."""
    return M >= 8 and N >= 8 and (K % 64 == 0 or not (a_kmajor or b_kmajor))


def _variant(a_kmajor: bool, splits: int, M: int = 0, N: int = 0, K: int = 0, b_kmajor: bool = True) -> int:
    if _VARIANT_ENV is not None:
        return int(_VARIANT_ENV)
    if splits == 1 and pp_eligible(M, N, K, a_kmajor, b_kmajor):
        # large products: 256 x 256 tile, per-phase DMA streaming, staggered
        # wave halves (1284 vs 1106 TF/s for the round-2 256 tile at 8192^3)
        return PP
    return 2 if (splits > 1 or not a_kmajor) else 10


def gemm(
    a: torch.Tensor,
    b: torch.Tensor,
    a_kmajor: bool = True,
    b_kmajor: bool = True,
    out_dtype: torch.dtype = torch.bfloat16,
    bias: Optional[torch.Tensor] = None,
    gelu: bool = False,
    want_z: bool = False,
    residual: Optional[torch.Tensor] = None,
    splits: int = 1,
    out: Optional[torch.Tensor] = None,
    variant: Optional[int] = None,
) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    """``(C, z)`` with ``C[m, n] = sum_k A(m, k) B(n, k)`` (+ epilogue).

    ``a`` is [M, K] if ``a_kmajor`` else [K, M]; ``b`` is [N, K] if
    ``b_kmajor`` else [K, N].  ``z`` is the GELU pre-activation (``want_z``).
    With ``splits > 1`` the K-slices' fp32 partials are summed inside the
    launch by the last slice to finish each tile (``ops/splitk.py``).
    """
    M = a.shape[0] if a_kmajor else a.shape[1]
    N = b.shape[0] if b_kmajor else b.shape[1]
    K = a.shape[1] if a_kmajor else a.shape[0]
    dev = a.device
    if variant is not None and variant & PP_ROWSPLIT:
        return _gemm_rowsplit(a, b, a_kmajor, b_kmajor, out_dtype, bias, gelu, want_z, residual, out, variant & ~PP_ROWSPLIT)
    force_il = variant is not None and bool(variant & GEMM_IL)
    if force_il:
        variant &= ~GEMM_IL
    if variant is not None and variant & PP_SK:  # stream-K: `splits` workgroups share the K-tile iterations
        if out is None:
            out = torch.empty((M, N), dtype=out_dtype, device=dev)
        z = torch.empty((M, N), dtype=torch.bfloat16, device=dev) if (gelu and want_z) else None
        ws = torch.empty(2 * splits * SK_SLAB, dtype=torch.float32, device=dev)
        _C().gemm(a, b, a_kmajor, b_kmajor, out, bias, gelu, z, residual, splits, variant, ws, counters(tiles_of(M, N), dev))
        return out, z
    if splits > 1:
        if out is None:
            out = torch.empty((M, N), dtype=out_dtype, device=dev)
        z = torch.empty((M, N), dtype=torch.bfloat16, device=dev) if (gelu and want_z) else None
        v = _variant(a_kmajor, splits) if variant is None else variant
        ws = torch.empty(splits * slab_elems(M, N, v), dtype=torch.float32, device=dev)
        if splits <= IN_LAUNCH_MAX_SPLITS or force_il:  # the last slice of each tile reduces it in the launch
            _C().gemm(a, b, a_kmajor, b_kmajor, out, bias, gelu, z, residual, splits, v, ws, counters(tiles_of(M, N), dev))
            return out, z
        if bias is not None or gelu or residual is not None:
            raise ValueError("a split-K GEMM with more than 4 slices has no epilogue")
        _C().gemm(a, b, a_kmajor, b_kmajor, ws, None, False, None, None, splits, v)
        if v & PP:  # the ping-pong kernels write row-major slabs
            _C().slab_sum(ws[: splits * M * N].view(splits, M * N), out.view(-1))
        else:
            _C().tile_slab_reduce(ws, splits, M, N, out, v)
        return out, z
    if out is None:
        out = torch.empty((M, N), dtype=out_dtype, device=dev)
    z = torch.empty((M, N), dtype=torch.bfloat16, device=dev) if (gelu and want_z) else None
    v = _variant(a_kmajor, 1, M, N, K, b_kmajor) if variant is None else variant
    _C().gemm(a, b, a_kmajor, b_kmajor, out, bias, gelu, z, residual, 1, v)
    return out, z


def rowsplit_rows(M: int, N: int) -> int:
    """Rows of the 256 x 256 launch of a row-split product: whole tile rows filling at
    most one wave of the 256 CUs (0 when the product has no second wave to trim)."""
    tiles_n = -(-N // 256)
    m1 = (256 // tiles_n) * 256 if tiles_n <= 256 else 0
    return m1 if 0 < m1 < M else 0


def _gemm_rowsplit(a, b, a_kmajor, b_kmajor, out_dtype, bias, gelu, want_z, residual, out, v):
    """A product whose 256 x 256 tiles spill a little past one wave (ViT fc2 input
    gradient / fc1 forward: 300 tiles on 256 CUs, 1.17 waves) as two launches over
    row ranges: the first ``rowsplit_rows`` rows on the 256 x 256 ping-pong kernel (one
    full wave), the rest on the 256 x 128 tile (its tail wave at half the work per
    workgroup).  Row slices of a k-major A / m-major A and of C, z, residual are views."""
    M = a.shape[0] if a_kmajor else a.shape[1]
    N = b.shape[0] if b_kmajor else b.shape[1]
    m1 = rowsplit_rows(M, N)
    if m1 == 0:
        return gemm(a, b, a_kmajor, b_kmajor, out_dtype, bias, gelu, want_z, residual, 1, out, v)
    if out is None:
        out = torch.empty((M, N), dtype=out_dtype, device=a.device)
    z = torch.empty((M, N), dtype=torch.bfloat16, device=a.device) if (gelu and want_z) else None
    for r0, r1, vv in ((0, m1, v), (m1, M, v | PP_N128)):
        aa = a[r0:r1] if a_kmajor else a[:, r0:r1]
        res = residual[r0:r1] if residual is not None else None
        _C().gemm(aa, b, a_kmajor, b_kmajor, out[r0:r1], bias, gelu, z[r0:r1] if z is not None else None, res, 1, vv)
    return out, z


def _wgrad(dy2: torch.Tensor, x2: torch.Tensor, dtype: torch.dtype, cfg: Optional[Tuple[int, int]] = None) -> torch.Tensor:
    """dW[n, k] = sum_m dy[m, n] x[m, k]: both operands m-major, split over m."""
    M, N = dy2.shape
    K = x2.shape[1]
    if cfg is None or not supported(N, K, M, False, False):  # e.g. a last batch of < 8 tokens
        return _product(dy2, x2, False, False, dtype, splits_for(N, K, M))
    v, sp = cfg
    return gemm(dy2, x2, False, False, out_dtype=dtype, splits=sp, variant=v)[0]


def _bias_grad(dy2: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    from p2pfl_amd.ops.fused import _fx

    return _fx().column_sum(dy2, dtype == torch.bfloat16).to(dtype)


def _rows(x: torch.Tensor) -> torch.Tensor:
    x2 = x.reshape(-1, x.shape[-1])
    if x2.stride(-1) != 1 or x2.stride(0) % 8 or x2.data_ptr() % 16:
        x2 = x2.contiguous()
    return x2


_NAT, _LIB = "native", "library"

# Native configurations tried per product at first use: (variant, split-K or, with
# PP_SK, stream-K grid).  From scripts/sk_sweep.py on the ViT-B/16 products
# (profiles/r6_vit_gemm_sweep.md): the N = 768 forward products and input gradients
# on the 256 x 128 ping-pong tile (150 whole tiles, no partial sums), the wider ones
# on the 256 x 256 ping-pong kernel (its 16x16x32 MFMA form where it wins) or the
# 128 x 128 single-buffer tile, the weight gradients (K = 6304 tokens, few output
# tiles) on the ping-pong kernel or the 4-stage ring at 6-8 K-slices.
# The stream-K schedule (PP_SK) is not offered: on every ViT product its partial-tile
# fix-up (256 KB fp32 per workgroup, ~15-18 us of chip-wide traffic) lost to the
# 256 x 128 tile's whole tiles (profiles/r6_vit_gemm_sweep.md, scripts/sk_anatomy.py).
def _fwd_cfgs(M: int, N: int, K: int):
    split = ((PP | PP_ROWSPLIT | PP_M16, 1), (PP | PP_ROWSPLIT, 1)) if rowsplit_rows(M, N) else ()
    return ((PP | PP_N128, 1), (PP | PP_N128 | PP_M16, 1), (PP | PP_M16, 1), (PP, 1), (PP, 2), (10, 1), (2, 1)) + split


def _dgrad_cfgs(M: int, N: int, K: int):
    split = ((PP | PP_ROWSPLIT | PP_M16, 1), (PP | PP_ROWSPLIT, 1)) if rowsplit_rows(M, N) else ()
    return ((PP | PP_N128, 1), (PP | PP_N128 | PP_M16, 1), (PP, 1), (PP, 2), (2, 1), (10, 1), (2, 3)) + split


# ping-pong at 3-4 slices reduces inside the launch (no slab-sum launch); at 6-8 slices
# through a separate slab_sum pass; unsplit tiles for short reductions (the ViT's
# class-token-only last block: K = batch rows)
_WGRAD_CFGS = ((PP, 6), (PP, 8), (PP, 4), (PP, 3), (PP | PP_M16, 6), (10, 6), (4096 | 2, 6), (2, 3),
                (PP | GEMM_IL, 6), (PP | GEMM_IL, 8), (4096 | 2 | GEMM_IL, 6), (2, 1), (PP, 1))


def _cfg_name(v: int, sp: int) -> str:
    return f"{_NAT}:{v}:{sp}"


def _cfg(choice: str) -> Tuple[int, int]:
    """(variant, splits) of a "native:v:s" choice."""
    _, v, sp = choice.split(":")
    return int(v), int(sp)


def _cfg_ok(v: int, sp: int, M: int, N: int, K: int, a_kmajor: bool, b_kmajor: bool, epilogue: bool) -> bool:
    """Configurations the kernels take for this product (no launch may fail)."""
    if not supported(M, N, K, a_kmajor, b_kmajor):
        return False
    il = bool(v & GEMM_IL)  # forced in-launch reduction: split-K only, takes every epilogue
    if il:
        if sp <= 1 or v & (PP_SK | PP_N128 | PP_ROWSPLIT):
            return False
        v &= ~GEMM_IL
        epilogue = False
    if v & PP and v & PP_SK:  # stream-K: any grid up to the iteration count, every epilogue
        return pp_eligible_any(M, N, K, a_kmajor, b_kmajor) and 1 <= sp <= sk_iters(M, N, K)
    if sp > 1 and K // sp < 256:
        return False
    if v & PP and v & (PP_N128 | PP_ROWSPLIT):  # the 256 x 128 tile (alone or as the row-split tail): no split-K
        return sp == 1 and pp_eligible_any(M, N, K, a_kmajor, b_kmajor) and (a_kmajor or not v & PP_ROWSPLIT
                                                                             or rowsplit_rows(M, N) % 8 == 0)
    if v & PP:
        return pp_eligible_any(M, N, K, a_kmajor, b_kmajor) and not (epilogue and sp > IN_LAUNCH_MAX_SPLITS)
    return not (epilogue and sp > IN_LAUNCH_MAX_SPLITS)


_ZERO_BIAS: dict = {}


def _zero_bias(n: int, device: torch.device) -> torch.Tensor:
    """A read-only fp32 zero vector of ``n`` (the bias operand of the fused GELU backward,
    whose pre-activation already includes the bias): allocated once per (n, device) outside
    a capture, so replayed steps carry no fill kernel (12 per ViT-B step before)."""
    key = (n, device)
    z = _ZERO_BIAS.get(key)
    if z is None:
        z = torch.zeros(n, dtype=torch.float32, device=device)
        if not (device.type == "cuda" and torch.cuda.is_current_stream_capturing()):
            _ZERO_BIAS[key] = z
    return z


class _LinearP(torch.autograd.Function):
    """``y = x W^T + b`` (or ``gelu(x W^T + b)``) whose three products -- forward,
    input gradient, weight gradient -- each run on the MFMA kernel configuration
    (``csrc/gemm*.hip``: tile, pipeline, split-K / stream-K) measured fastest for its
    own shape (``_plan``).  The forward's bias / GELU ride in the kernel's epilogue
    (which also keeps the pre-activation for the backward); the bias gradient is the
    column-sum kernel, or comes out of the fused GELU backward."""

    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda")  # operands cast here, the bias keeps its dtype (no cast kernels)
    def forward(ctx, x, w, b, gelu, plan, keep_z=True):
        fwd = plan[0]
        x2 = _rows(x.to(torch.bfloat16))
        wc = w.to(torch.bfloat16).contiguous()
        v, sp = _cfg(fwd)
        pre = gb = None
        if not gelu:
            y = gemm(x2, wc, bias=b, variant=v, splits=sp)[0]  # the epilogue reads an fp32 or a bf16 bias
        else:
            # the pre-activation (bias included) is kept only for a backward: an evaluation
            # forward skips its store (M x N bf16, as many bytes as the output itself)
            y, pre = gemm(x2, wc, bias=b, gelu=True, want_z=keep_z, variant=v, splits=sp)
            gb = _zero_bias(w.shape[0], x.device) if keep_z else None
        STATS["native"] += 1
        ctx.save_for_backward(x2, wc, pre, gb)
        ctx.gelu, ctx.plan = gelu, plan
        ctx.w_dtype = w.dtype
        ctx.b_dtype = b.dtype if b is not None else None
        ctx.bias = b
        from p2pfl_amd.ops.fused import defer_scope

        ctx.defer = defer_scope()  # recorded on the caller's thread (see ops.fused.deferred_param_grads)
        ctx.xshape = x.shape
        return y.view(*x.shape[:-1], w.shape[0])

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, dy):
        from p2pfl_amd.ops.fused import _fx

        x2, w, pre, gb = ctx.saved_tensors
        _, dg, wg = ctx.plan
        from p2pfl_amd.ops.fused import defer_colsum, defer_grad

        dz = _rows(dy.to(torch.bfloat16))
        db = None
        want_db = ctx.b_dtype is not None and ctx.needs_input_grad[2]
        d = ctx.defer if ctx.defer is not None and ctx.defer.open else None
        if ctx.gelu and want_db and d is not None:  # the column reduction runs at the end of the backward
            dz, pdb = _fx().bias_gelu_bwd_parts(dz, pre, gb)
            if not defer_grad(d, ctx.bias, pdb):
                db = pdb.sum(0)
        elif ctx.gelu:
            dz, db = _fx().bias_gelu_bwd(dz, pre, gb)  # dz = dy * gelu'(pre), db = column sums of dz
        elif want_db and d is not None and defer_colsum(d, ctx.bias, dz):
            pass  # partials and reduction both run batched after the backward
        elif want_db and d is not None and dz.shape[0] > 0:
            part = _fx().column_sum_parts(dz)
            if not defer_grad(d, ctx.bias, part):
                db = part.sum(0)
        elif want_db:
            db = _bias_grad(dz, ctx.b_dtype)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            v, sp = _cfg(dg)
            if supported(dz.shape[0], w.shape[1], w.shape[0], True, False):
                dx = gemm(dz, w, True, False, splits=sp, variant=v)[0].view(ctx.xshape)
            else:
                dx = _product(dz, w, True, False, torch.bfloat16).view(ctx.xshape)
        if ctx.needs_input_grad[1]:
            dw = _wgrad(dz, x2, ctx.w_dtype, _cfg(wg))
        if db is not None and ctx.b_dtype is not None:
            db = db.to(ctx.b_dtype)
        return dx, dw, db if (ctx.b_dtype is not None and ctx.needs_input_grad[2]) else None, None, None, None


# P2PFL_NATIVE_GEMM: "native" / "auto" (default): every bf16 Linear product on the
# hand-written kernels; "library": hipBLASLt (torch.mm / F.linear) -- an A/B
# measurement knob only, never chosen at run time.
_POLICY = autotune.policy("P2PFL_NATIVE_GEMM")
_FALLBACK_CFG = _cfg_name(0, 1)  # the 128 x 128 double-buffer tile: takes every supported shape


def _plan(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor], gelu: bool) -> Tuple[str, str, str]:
    """(forward, input gradient, weight gradient) kernel configurations: each product
    timed once per shape over the native configurations it admits (HIP events,
    ops/autotune.py) and the fastest remembered -- tile shape (256 x 256 / 256 x 128
    ping-pong, 128 x 128), MFMA form, split-K or stream-K
    (profiles/r6_vit_gemm_sweep.md).  Inside a capture nothing can be timed: an
    unseen product takes a configuration every shape admits."""
    grad = torch.is_grad_enabled() and (x.requires_grad or w.requires_grad)
    M = x.numel() // x.shape[-1]
    N, K = w.shape
    keys = (("linear_fwd", M, N, K, bool(gelu), bias is not None), ("linear_dgrad", M, N, K), ("linear_wgrad", M, N, K))
    got = [autotune._CHOICE.get(k) for k in keys]
    if got[0] is not None and (not grad or (got[1] is not None and got[2] is not None)):
        return (got[0], got[1] or _FALLBACK_CFG, got[2] or _FALLBACK_CFG)  # steady state: no allocation
    if torch.cuda.is_current_stream_capturing():
        return tuple(g or _FALLBACK_CFG for g in got)  # type: ignore[return-value]
    x2 = x.detach().reshape(M, K).to(torch.bfloat16)
    wd = w.detach().to(torch.bfloat16).contiguous()
    bd = bias.detach() if bias is not None else None
    epi = gelu or bias is not None
    fwd_c = [(_cfg_name(v, sp), (lambda v=v, sp=sp: gemm(x2, wd, bias=bd, gelu=gelu, want_z=gelu and grad, variant=v, splits=sp)))
             for v, sp in _fwd_cfgs(M, N, K) if _cfg_ok(v, sp, M, N, K, True, True, epi)]
    fwd = autotune.choose(keys[0], fwd_c or [(_FALLBACK_CFG, lambda: None)])
    if not grad:
        return fwd, _FALLBACK_CFG, _FALLBACK_CFG
    dy = torch.randn(M, N, device=x.device).to(torch.bfloat16)
    dg_c = [(_cfg_name(v, sp), (lambda v=v, sp=sp: gemm(dy, wd, True, False, splits=sp, variant=v)))
            for v, sp in _dgrad_cfgs(M, K, N) if _cfg_ok(v, sp, M, K, N, True, False, False)]
    dg = autotune.choose(keys[1], dg_c or [(_FALLBACK_CFG, lambda: None)])
    wg_c = [(_cfg_name(v, sp), (lambda v=v, sp=sp: _wgrad(dy, x2, torch.bfloat16, (v, sp))))
            for v, sp in _WGRAD_CFGS if _cfg_ok(v, sp, N, K, M, False, False, False)]
    wg = autotune.choose(keys[2], wg_c or [(_FALLBACK_CFG, lambda: None)])
    return fwd, dg, wg


def _bf16_call(x: torch.Tensor) -> bool:
    """A bf16 product: a bf16 input, or an fp32 one under bf16 autocast (an fp32
    product outside autocast keeps fp32 math)."""
    return x.dtype == torch.bfloat16 or (
        x.dtype == torch.float32 and torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16)


def _ok(x: torch.Tensor, w: torch.Tensor) -> bool:
    """bf16 products on the GPU whose shapes the kernels take."""
    from p2pfl_amd.ops import _gpu

    return _gpu(x) and _bf16_call(x) and w.shape[0] % 8 == 0 and w.shape[1] % 8 == 0 and x.shape[-1] == w.shape[1]


def _library(x: torch.Tensor) -> bool:
    """hipBLASLt for this call: the A/B knob, or a bf16 product the kernels refuse
    (counted, and refused under P2PFL_STRICT_NATIVE)."""
    if _POLICY == _LIB:
        return True
    torch_fallback(f"Linear {tuple(x.shape)}")
    return True


def linear(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``F.linear`` with its three products on the MFMA GEMM (per-shape kernel configuration)."""
    if _POLICY != _LIB and _ok(x, weight):
        return _LinearP.apply(x, weight, bias, False, _plan(x, weight, bias, False))
    if x.is_cuda and (_POLICY == _LIB or _bf16_call(x)) and _library(x):
        from p2pfl_amd.ops.fused import linear as linear_blas

        return linear_blas(x, weight, bias)
    return F.linear(x, weight, bias)


def linear_gelu(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor) -> torch.Tensor:
    """``gelu(F.linear(x, weight, bias))`` (exact erf GELU), fused epilogue."""
    if _POLICY != _LIB and _ok(x, weight):
        grad = torch.is_grad_enabled() and (x.requires_grad or weight.requires_grad or bias.requires_grad)
        return _LinearP.apply(x, weight, bias, True, _plan(x, weight, bias, True), grad)
    if x.is_cuda and (_POLICY == _LIB or _bf16_call(x)) and _library(x):
        from p2pfl_amd.ops.fused import bias_gelu, linear as linear_blas

        return bias_gelu(linear_blas(x, weight, None), bias)
    return F.gelu(F.linear(x, weight, bias))
