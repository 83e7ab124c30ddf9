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


def _product(a, b, a_kmajor, b_kmajor, dtype, splits=1):
    """One Linear product on the MFMA kernel, or torch for shapes it does not take."""
    M = a.shape[0] if a_kmajor else a.shape[1]
    N = b.shape[0] if b_kmajor else b.shape[1]
    K = a.shape[1] if a_kmajor else a.shape[0]
    if supported(M, N, K, a_kmajor, b_kmajor):
        return gemm(a, b, a_kmajor, b_kmajor, out_dtype=dtype, splits=splits)[0]
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
        if splits <= IN_LAUNCH_MAX_SPLITS:  # the last slice of each tile reduces it in the launch
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


def _wgrad(dy2: torch.Tensor, x2: torch.Tensor, dtype: torch.dtype, cfg: Optional[Tuple[int, int]] = None) -> torch.Tensor:
    """dW[n, k] = sum_m dy[m, n] x[m, k]: both operands m-major, split over m."""
    M, N = dy2.shape
    K = x2.shape[1]
    if cfg is None:
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

# Native configurations tried per product at first use: (variant, split-K).
# From scripts/vit_gemm_sweep.py on the ViT-B/16 products (profiles/r5_vit_gemm_sweep.md):
# the forward products by the ping-pong kernel (its 16x16x32 form on qkv / proj /
# patch) or the 128 x 128 single-buffer tile (fc1), the input gradients by the
# ping-pong kernel (2 in-launch slices when N = 768) or the 128 x 128 double
# buffer, the weight gradients (K = 6304 tokens, few output tiles) by the
# ping-pong kernel or the 4-stage ring at 6-8 slices.
_FWD_CFGS = ((PP | PP_M16, 1), (PP, 1), (PP, 2), (2, 1), (10, 1))
_DGRAD_CFGS = ((PP, 1), (PP, 2), (2, 1), (10, 1), (2, 3), (10, 2))
_WGRAD_CFGS = ((PP, 6), (PP, 8), (10, 6), (4096 | 2, 6), (2, 3))


def _cfg_name(v: int, sp: int) -> str:
    return f"{_NAT}:{v}:{sp}"


def _cfg(choice: str) -> Tuple[int, int]:
    """(variant, splits) of a "native:v:s" choice."""
    _, v, sp = choice.split(":")
    return int(v), int(sp)


def _cfg_ok(v: int, sp: int, M: int, N: int, K: int, a_kmajor: bool, b_kmajor: bool, epilogue: bool) -> bool:
    """Configurations the kernels take for this product (no launch may fail)."""
    if not supported(M, N, K, a_kmajor, b_kmajor) or (sp > 1 and K // sp < 256):
        return False
    if v & PP:
        return pp_eligible_any(M, N, K, a_kmajor, b_kmajor) and not (epilogue and sp > IN_LAUNCH_MAX_SPLITS)
    return not (epilogue and sp > IN_LAUNCH_MAX_SPLITS)


class _LinearP(torch.autograd.Function):
    """``y = x W^T + b`` (or ``gelu(x W^T + b)``) whose three products -- forward,
    input gradient, weight gradient -- each run on the path measured fastest for
    its own shape (``plan``): the MFMA kernel of ``csrc/gemm*.hip`` or hipBLASLt.
    The forward's bias / GELU ride in the native epilogue (which also keeps the
    pre-activation for the backward), or in the fused bias+GELU kernel after a
    bias-free hipBLASLt GEMM; the bias gradient is the column-sum kernel, or comes
    out of the fused GELU backward."""

    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda")  # operands cast here, the bias keeps its dtype (no cast kernels)
    def forward(ctx, x, w, b, gelu, plan):
        from p2pfl_amd.ops.fused import _fx

        fwd = plan[0]
        x2 = _rows(x.to(torch.bfloat16))
        wc = w.to(torch.bfloat16).contiguous()
        pre = gb = None
        nat = fwd.startswith(_NAT)
        v, sp = _cfg(fwd) if ":" in fwd else (None, 1)
        if not gelu:
            # the native epilogue reads an fp32 or a bf16 bias; hipBLASLt needs x's dtype
            y = gemm(x2, wc, bias=b, variant=v, splits=sp)[0] if nat else F.linear(x2, wc, b.to(torch.bfloat16) if b is not None else None)
        elif nat:
            y, pre = gemm(x2, wc, bias=b, gelu=True, want_z=True, variant=v, splits=sp)  # pre-activation includes the bias
            gb = torch.zeros(w.shape[0], dtype=torch.float32, device=x.device)
        else:
            pre = torch.mm(x2, wc.t())  # bias-free; the GELU kernel adds it (fp32: fc1.bias is an fp32 parameter)
            gb = b if (b.dtype == torch.float32 and b.is_contiguous()) else b.float().contiguous()
            y = _fx().bias_gelu_fwd(pre, gb)
        ctx.save_for_backward(x2, wc, pre, gb)
        ctx.gelu, ctx.plan = gelu, plan
        ctx.w_dtype = w.dtype
        ctx.b_dtype = b.dtype if b is not None else None
        ctx.xshape = x.shape
        return y.view(*x.shape[:-1], w.shape[0])

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, dy):
        from p2pfl_amd.ops.fused import _fx, _wgrad as wgrad_blas

        x2, w, pre, gb = ctx.saved_tensors
        _, dg, wg = ctx.plan
        dz = _rows(dy.to(torch.bfloat16))
        db = None
        if ctx.gelu:
            dz, db = _fx().bias_gelu_bwd(dz, pre, gb)  # dz = dy * gelu'(pre), db = column sums of dz
        elif ctx.b_dtype is not None and ctx.needs_input_grad[2]:
            db = _bias_grad(dz, ctx.b_dtype)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            if dg.startswith(_NAT):
                v, sp = _cfg(dg) if ":" in dg else (None, 1)
                dx = gemm(dz, w, True, False, splits=sp, variant=v)[0] if v is not None else _product(dz, w, True, False, torch.bfloat16)
            else:
                dx = torch.mm(dz, w)
            dx = dx.view(ctx.xshape)
        if ctx.needs_input_grad[1]:
            if wg.startswith(_NAT):
                dw = _wgrad(dz, x2, ctx.w_dtype, _cfg(wg) if ":" in wg else None)
            else:
                dw = wgrad_blas(dz, x2).to(ctx.w_dtype)
        if db is not None and ctx.b_dtype is not None:
            db = db.to(ctx.b_dtype)
        return dx, dw, db if (ctx.b_dtype is not None and ctx.needs_input_grad[2]) else None, None, None


# "native" | "library" | "auto" (measured per product and shape, ops/autotune.py); env P2PFL_NATIVE_GEMM.
# The library side is hipBLASLt (torch.mm / F.linear) plus the fused bias+GELU kernel.
_POLICY = autotune.policy("P2PFL_NATIVE_GEMM")


def _plan(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor], gelu: bool) -> Tuple[str, str, str]:
    """(forward, input gradient, weight gradient): each product timed once per
    shape on both paths (HIP events, ops/autotune.py) and the winner remembered.
    Deciding per product, not per layer, keeps e.g. a native weight gradient that
    beats hipBLASLt even where the library forward is faster
    (profiles/r4_gemm_w4.md: native wins all four ViT weight gradients)."""
    if _POLICY == _NAT:
        return _NAT, _NAT, _NAT
    grad = torch.is_grad_enabled() and (x.requires_grad or w.requires_grad)
    M = x.numel() // x.shape[-1]
    N, K = w.shape
    keys = (("linear_fwd", M, N, K, bool(gelu), bias is not None), ("linear_dgrad", M, N, K), ("linear_wgrad", M, N, K))
    got = [autotune._CHOICE.get(k) for k in keys]
    if got[0] is not None and (not grad or (got[1] is not None and got[2] is not None)):
        return (got[0], got[1], got[2]) if grad else (got[0], _LIB, _LIB)  # steady state: no allocation
    if torch.cuda.is_current_stream_capturing():  # nothing can be timed inside a capture
        return tuple(g or _NAT for g in got)  # type: ignore[return-value]
    from p2pfl_amd.ops.fused import _fx, _wgrad as wgrad_blas

    x2 = x.detach().reshape(M, K).to(torch.bfloat16)
    wd = w.detach().to(torch.bfloat16).contiguous()
    bd = bias.detach() if bias is not None else None
    bd16 = bd.to(torch.bfloat16) if bd is not None else None
    g32 = bd.float().contiguous() if bd is not None else None

    def fwd_library():
        if gelu:
            _fx().bias_gelu_fwd(torch.mm(x2, wd.t()), g32)
        else:
            F.linear(x2, wd, bd16)

    epi = gelu or bias is not None
    fwd_c = [(_cfg_name(v, sp), (lambda v=v, sp=sp: gemm(x2, wd, bias=bd, gelu=gelu, want_z=gelu and grad, variant=v, splits=sp)))
             for v, sp in _FWD_CFGS if _cfg_ok(v, sp, M, N, K, True, True, epi)]
    fwd = autotune.choose(keys[0], fwd_c + [(_LIB, fwd_library)])
    if not grad:
        return fwd, _LIB, _LIB
    dy = torch.randn(M, N, device=x.device).to(torch.bfloat16)
    dg_c = [(_cfg_name(v, sp), (lambda v=v, sp=sp: gemm(dy, wd, True, False, splits=sp, variant=v)))
            for v, sp in _DGRAD_CFGS if _cfg_ok(v, sp, M, K, N, True, False, False)]
    dg = autotune.choose(keys[1], dg_c + [(_LIB, lambda: torch.mm(dy, wd))])
    wg_c = [(_cfg_name(v, sp), (lambda v=v, sp=sp: _wgrad(dy, x2, torch.bfloat16, (v, sp))))
            for v, sp in _WGRAD_CFGS if _cfg_ok(v, sp, N, K, M, False, False, False)]
    wg = autotune.choose(keys[2], wg_c + [(_LIB, lambda: wgrad_blas(dy, x2))])
    return fwd, dg, wg


def _ok(x: torch.Tensor, w: torch.Tensor) -> bool:
    """bf16 products on the GPU: a bf16 input, or an fp32 one under bf16 autocast
    (an fp32 product outside autocast keeps fp32 math on hipBLASLt)."""
    from p2pfl_amd.ops import _gpu

    bf16 = x.dtype == torch.bfloat16 or (
        x.dtype == torch.float32 and torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16)
    return _gpu(x) and bf16 and w.shape[0] % 8 == 0 and w.shape[1] % 8 == 0 and x.shape[-1] == w.shape[1]


def linear(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``F.linear`` with each of its three products on the MFMA GEMM or hipBLASLt, per measured shape."""
    if _POLICY != _LIB and _ok(x, weight):
        return _LinearP.apply(x, weight, bias, False, _plan(x, weight, bias, False))
    if x.is_cuda:
        from p2pfl_amd.ops.fused import linear as linear_blas

        return linear_blas(x, weight, bias)
    return F.linear(x, weight, bias)


def linear_gelu(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor) -> torch.Tensor:
    """``gelu(F.linear(x, weight, bias))`` (exact erf GELU), fused epilogue."""
    if _POLICY != _LIB and _ok(x, weight):
        return _LinearP.apply(x, weight, bias, True, _plan(x, weight, bias, True))
    if x.is_cuda:
        from p2pfl_amd.ops.fused import bias_gelu, linear as linear_blas

        return bias_gelu(linear_blas(x, weight, None), bias)
    return F.gelu(F.linear(x, weight, bias))
