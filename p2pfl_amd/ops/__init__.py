"""Hand-written HIP/CDNA4 kernels (``csrc/*.hip``, extension ``p2pfl_amd._C``).

Every op has a plain-torch implementation used for CPU tensors (the control
plane and the CPU test-suite run without a GPU) and as the fp32 reference in
numerics tests.  For GPU tensors the HIP kernel is mandatory: if the extension
is missing on a GPU box the call raises instead of silently falling back, so a
"passing" GPU run always exercised the native path.
"""

from __future__ import annotations

import importlib
import os
from typing import Tuple, List, Optional, Sequence

import torch

_ext = None
_ext_error: Optional[BaseException] = None


def _load():
    global _ext, _ext_error
    if _ext is None and _ext_error is None:
        try:
            _ext = importlib.import_module("p2pfl_amd._C")
        except BaseException as e:  # ImportError, OSError (missing HIP runtime), ...
            _ext_error = e
    return _ext


def available() -> bool:
    return _load() is not None


def ext():
    """The native extension; raises loudly if it was not built."""
    m = _load()
    if m is None:
        raise RuntimeError(
            "p2pfl_amd native extension (p2pfl_amd._C) is not available: "
            f"{_ext_error!r}. Build it with `python setup.py build_ext --inplace` "
            "(PYTORCH_ROCM_ARCH=gfx950)."
        )
    return m


def _gpu(t: torch.Tensor) -> bool:
    return t.is_cuda and os.environ.get("P2PFL_FORCE_TORCH_OPS") != "1"


# ----------------------------------------------------------------------------
# aggregation
# ----------------------------------------------------------------------------
def normalized_weights(weights: Sequence[float]) -> List[float]:
    total = float(sum(weights))
    if total <= 0:
        return [1.0 / len(weights)] * len(weights)
    return [float(w) / total for w in weights]


def fedavg_weights(weights: Sequence[float]) -> Tuple[List[float], float]:
    """(per-input weights, final scale) of a weighted mean: ``sum w_i x_i / sum w_i``
    is computed as raw-weight fp32 FMAs followed by ONE multiply by ``1 / sum w``,
    so it can be folded in several pieces (running sum) with bitwise-equal
    results.  All-zero weights fall back to the plain mean."""
    total = float(sum(weights))
    if total <= 0:
        return [1.0] * len(weights), 1.0 / len(weights)
    return [float(w) for w in weights], 1.0 / total


def weighted_sum_into(
    out: torch.Tensor,
    flats: Sequence[torch.Tensor],
    weights: Sequence[float],
    acc_in: Optional[torch.Tensor] = None,
    scale: float = 1.0,
) -> torch.Tensor:
    """``out = scale * (acc_in + sum_i weights[i] * flats[i])`` in fp32 (``acc_in``
    None = 0; it may be ``out`` itself).  One fused kernel on the GPU; the same
    operation sequence on the CPU, so pieces folded separately equal one call."""
    if not flats and acc_in is None:
        raise ValueError("no inputs")
    dev_t = flats[0] if flats else out
    if not _gpu(dev_t):
        acc = acc_in.clone() if acc_in is not None else torch.zeros(out.shape, dtype=torch.float32, device=out.device)
        for f, w in zip(flats, weights):
            acc.add_(f.to(acc.device, torch.float32), alpha=float(w))
        if scale != 1.0:
            acc.mul_(scale)
        out.copy_(acc)
        return out
    dev = out.device
    ok = (torch.float32, torch.bfloat16)
    srcs = [f if (f.device == dev and f.dtype in ok and f.is_contiguous() and f.data_ptr() % 16 == 0)
            else f.to(dev, torch.float32).contiguous() for f in flats]
    ext().weighted_sum(srcs, [float(w) for w in weights], out, acc_in, float(scale))
    return out


def weighted_average_reference(flats: Sequence[torch.Tensor], weights: Sequence[float]) -> torch.Tensor:
    w, scale = fedavg_weights(weights)
    acc = torch.zeros_like(flats[0], dtype=torch.float32)
    for f, wi in zip(flats, w):
        acc.add_(f.float(), alpha=wi)
    return acc.mul_(scale)


def weighted_average(
    flats: Sequence[torch.Tensor],
    weights: Sequence[float],
    out: Optional[torch.Tensor] = None,
    out_dtype: torch.dtype = torch.float32,
) -> torch.Tensor:
    """``sum_i w_i * flats[i] / sum_i w_i`` with fp32 accumulation (one fused kernel on GPU).

    Inputs may be fp32 or bf16 arenas in any mix (bf16 ones come from peers on
    the bf16 wire option) -- the kernel widens them in registers, no
    conversion pass; the result is fp32 (default) or bf16.
    """
    if len(flats) == 0:
        raise ValueError("no inputs")
    n = flats[0].numel()
    for f in flats:
        if f.numel() != n:
            raise ValueError("inputs differ in size")
    if out is not None:
        out_dtype = out.dtype
    w, scale = fedavg_weights(weights)
    if not _gpu(flats[0]):
        res = weighted_average_reference(flats, weights)
        if out is not None:
            out.copy_(res)
            return out
        return res.to(out_dtype)
    dev = flats[0].device
    if out_dtype == torch.bfloat16 and len(flats) > 16:
        res = weighted_average(flats, weights)  # fp32 partial sums, then one cast
        if out is None:
            return res.to(torch.bfloat16)
        out.copy_(res)
        return out
    if out is None:
        out = torch.empty(n, dtype=out_dtype, device=dev)
    return weighted_sum_into(out, flats, w, None, scale)


# ----------------------------------------------------------------------------
# optimizers (whole-arena, in place)
# ----------------------------------------------------------------------------
def adam_step_reference(p, g, m, v, lr, beta1, beta2, eps, weight_decay, step, decoupled=False):
    if weight_decay != 0:
        if decoupled:
            p.mul_(1 - lr * weight_decay)
        else:
            g = g + weight_decay * p
    m.mul_(beta1).add_(g, alpha=1 - beta1)
    v.mul_(beta2).addcmul_(g, g, value=1 - beta2)
    bc1 = 1 - beta1**step
    bc2 = 1 - beta2**step
    denom = (v.sqrt() / (bc2**0.5)).add_(eps)
    p.addcdiv_(m, denom, value=-lr / bc1)


def adam_step(p, g, m, v, *, lr, beta1, beta2, eps, weight_decay, step, decoupled=False, p_bf16=None):
    """In-place Adam/AdamW over flat fp32 buffers (optionally also writes a bf16 copy of p)."""
    if not _gpu(p):
        adam_step_reference(p, g, m, v, lr, beta1, beta2, eps, weight_decay, step, decoupled)
        if p_bf16 is not None:
            p_bf16.copy_(p)
        return
    ext().adam_step(p, g, m, v, p_bf16, float(lr), float(beta1), float(beta2), float(eps), float(weight_decay), int(step), bool(decoupled))


def sgd_step_reference(p, g, buf, lr, momentum, dampening, weight_decay, nesterov, first_step):
    if weight_decay != 0:
        g = g + weight_decay * p
    if momentum != 0:
        if first_step:
            buf.copy_(g)
        else:
            buf.mul_(momentum).add_(g, alpha=1 - dampening)
        g = g + momentum * buf if nesterov else buf
    p.add_(g, alpha=-lr)


def sgd_step(p, g, buf, *, lr, momentum=0.0, dampening=0.0, weight_decay=0.0, nesterov=False, first_step=False, p_bf16=None):
    if not _gpu(p):
        sgd_step_reference(p, g, buf, lr, momentum, dampening, weight_decay, nesterov, first_step)
        if p_bf16 is not None:
            p_bf16.copy_(p)
        return
    ext().sgd_step(p, g, buf, p_bf16, float(lr), float(momentum), float(dampening), float(weight_decay), bool(nesterov), bool(first_step))


# ----------------------------------------------------------------------------
# multi-tensor optimizers (mixed-precision learners: per-tensor grads, flat state)
# ----------------------------------------------------------------------------
def _mt_reference(step_fn, p, states, pbf, table, grads):
    for (off, n, flags), g in zip(table, grads):
        if g is None:
            continue
        view = lambda t: t[off : off + n]  # noqa: E731
        step_fn(view(p), g.reshape(-1).float(), *[view(s) if s is not None else None for s in states])
        if pbf is not None and flags & 2:
            if flags & 4:  # channels-last shadow region
                i, hw = (flags >> 8) & 0xFFFFFF, (flags >> 32) & 0xFFFFFF
                view(pbf).view(-1, hw, i).copy_(view(p).view(-1, i, hw).transpose(1, 2))
            else:
                view(pbf).copy_(view(p))


def adam_mt_step(p, m, v, grads, mt, *, lr, beta1, beta2, eps, weight_decay, step, decoupled=False, p_bf16=None, gtab=None, t_dev=None):
    """Adam/AdamW for tensors whose grads live outside the arena (``mt``: :class:`~p2pfl_amd.learning.optim.MTTables`).

    ``gtab`` (device int64 [T]) replaces ``grads`` by a persistent table of
    gradient addresses and ``t_dev`` (device int32 [1]) supplies the step
    count: together they make the launch replayable inside a HIP graph.
    """
    if not _gpu(p):
        _mt_reference(
            lambda pp, g, mm, vv: adam_step_reference(pp, g, mm, vv, lr, beta1, beta2, eps, weight_decay, step, decoupled),
            p, (m, v), p_bf16, mt.table, grads,
        )
        return
    ext().adam_mt_step(
        p, m, v, p_bf16, mt.tens, mt.chunks, list(grads), mt.numels, mt.grad_bf16, mt.grad_cl,
        float(lr), float(beta1), float(beta2), float(eps), float(weight_decay), int(step), bool(decoupled), gtab, t_dev,
    )


def sgd_mt_step(p, buf, grads, mt, *, lr, momentum=0.0, dampening=0.0, weight_decay=0.0, nesterov=False, first_step=False, p_bf16=None, gtab=None):
    if not _gpu(p):
        _mt_reference(
            lambda pp, g, b: sgd_step_reference(pp, g, b, lr, momentum, dampening, weight_decay, nesterov, first_step),
            p, (buf,), p_bf16, mt.table, grads,
        )
        return
    ext().sgd_mt_step(
        p, buf, p_bf16, mt.tens, mt.chunks, list(grads), mt.numels, mt.grad_bf16, mt.grad_cl,
        float(lr), float(momentum), float(dampening), float(weight_decay), bool(nesterov), bool(first_step), gtab,
    )


# ----------------------------------------------------------------------------
# fused transformer / classifier ops (csrc/fused_ops.hip)
# ----------------------------------------------------------------------------
from p2pfl_amd.ops.fused import (  # noqa: E402
    add_layer_norm,
    add_layer_norm_reference,
    attention_qkv,
    attention_qkv_reference,
    bias_gelu,
    bias_gelu_reference,
    embed_tokens,
    layer_norm,
    layer_norm_reference,
    patchify_u8,
    softmax_xent,
    softmax_xent_reference,
)
from p2pfl_amd.ops.fused import linear as linear_blas  # noqa: E402,F401  (hipBLASLt comparison path)
from p2pfl_amd.ops.gemm import gemm, gemm_reference, linear, linear_gelu  # noqa: E402,F401
from p2pfl_amd.ops.conv import conv2d  # noqa: E402,F401
