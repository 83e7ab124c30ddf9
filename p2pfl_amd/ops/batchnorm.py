"""Fused BatchNorm (+ residual add) (+ ReLU) on channels-last activations (``csrc/batchnorm.hip``).

ResNet blocks (BASELINE.json configs 3 and 5) spend their non-convolution time
in ``BatchNorm2d -> (+ shortcut) -> ReLU``: three elementwise-class passes
forward and three backward on PyTorch-ROCm.  :func:`batch_norm_act` runs the
whole chain as one column-statistics pass plus one apply pass in each
direction, reading the NHWC activation as an ``[N*H*W, C]`` matrix.

Semantics equal ``act(F.batch_norm(x, ...) + residual)``: biased batch
variance for normalisation, unbiased variance and ``momentum`` for the running
statistics, ``num_batches_tracked`` incremented on the device.  Eval mode
uses the running statistics.  CPU tensors, NCHW-contiguous tensors, channel
counts not divisible by 8 and ``momentum=None`` use the plain PyTorch chain.
"""

from __future__ import annotations

import os
from typing import Optional

import torch
import torch.nn.functional as F
from torch import nn


# host-side counters of the extra passes the backward had to insert
STATS = {"dy_cast": 0, "dy_relayout": 0, "dy_pairs": 0}
# statistics + finalize as one launch for eligible bf16 shapes (P2PFL_BN_FUSED_STATS=1).  Off by
# default: per call it is 8.4 us against 4.9 + 4.9 us for the two launches, but the ResNet-18 /
# ResNet-50 rounds measured 3.5 % / 2.5 % slower with it (profiles/r3_bn_stats_finalize.md).
_FUSED_STATS = os.environ.get("P2PFL_BN_FUSED_STATS", "0") == "1"


def _bx():
    from p2pfl_amd.ops import ext

    return ext().bn


def _counter(x2: torch.Tensor):
    """Arrival counter of the statistics + finalize kernel (one launch instead of
    two, csrc/batchnorm.hip) when the [M, C] activation is eligible, else None."""
    if x2.dtype != torch.bfloat16 or not _FUSED_STATS or _bx().fused_rows(x2.shape[0], x2.shape[1]) <= 0:
        return None
    from p2pfl_amd.ops import splitk

    return splitk.counters(1, x2.device)


def _nhwc_2d(t: torch.Tensor) -> torch.Tensor:
    """[N, C, H, W] channels-last tensor -> its [N*H*W, C] storage view."""
    return t.permute(0, 2, 3, 1).reshape(-1, t.shape[1])


def _from_2d(t2: torch.Tensor, shape) -> torch.Tensor:
    n, c, h, w = shape
    return t2.view(n, h, w, c).permute(0, 3, 1, 2)


def batch_norm_act_reference(x, weight, bias, running_mean, running_var, training, momentum, eps, residual=None, relu=True):
    """Plain PyTorch definition (also the CPU / fallback path)."""
    y = F.batch_norm(x, running_mean, running_var, weight, bias, training, momentum, eps)
    if residual is not None:
        y = y + residual
    return torch.relu(y) if relu else y


def _outputs(ctx, y2, shape, fork: bool):
    """The NCHW view of y2, or with ``fork`` that view and an alias of it: two autograd
    outputs for the two consumers of a residual block's input (its first convolution
    and its shortcut), whose gradients the backward then sums inside the BN kernels
    instead of autograd adding them in a separate pass."""
    y = _from_2d(y2, shape)
    if not fork:
        return y
    ctx.set_materialize_grads(False)  # an unused alias brings None, not a zero-filled gradient
    return y, y.view_as(y)


def _grads(dy, dy2):
    """(dy, dy2) of a forked output with None for a branch that sent no gradient."""
    if dy is None:
        return dy2, None
    return dy, dy2


class _BatchNormAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, residual, running_mean, running_var, nbt, momentum, eps, relu, fork=False):
        shape = x.shape
        x2 = _nhwc_2d(x)
        r2 = _nhwc_2d(residual.to(x.dtype)) if residual is not None else None
        y2, mean, rstd = _bx().fwd_train(x2, weight, bias, r2, running_mean, running_var, nbt, float(momentum), float(eps), bool(relu),
                                         _counter(x2))
        ctx.save_for_backward(x2, y2, weight, mean, rstd)
        ctx.shape, ctx.relu, ctx.has_res = shape, bool(relu), residual is not None
        ctx.res_dtype = residual.dtype if residual is not None else None
        return _outputs(ctx, y2, shape, fork)

    @staticmethod
    def backward(ctx, dy, dy2=None):
        return _bn_backward(ctx, *_grads(dy, dy2)) + (None,) * 7


def _bn_backward(ctx, dy, dy2=None):
    """(dx, dweight, dbias, dresidual) of act(bn(x) [+ residual]) from the saved x2, y2, weight,
    mean, rstd; ``dy2``: the gradient of the forked alias output, summed with dy in the kernels."""
    x2, y2, weight, mean, rstd = ctx.saved_tensors
    if dy is None:  # neither branch used the output
        return None, None, None, None

    def prep(g):
        if g.dtype != x2.dtype:
            STATS["dy_cast"] += 1
            g = g.to(x2.dtype)
        if not g.is_contiguous(memory_format=torch.channels_last):
            STATS["dy_relayout"] += 1
            g = g.contiguous(memory_format=torch.channels_last)
        return _nhwc_2d(g)

    if dy2 is not None:
        STATS["dy_pairs"] += 1
    out = _bx().bwd(prep(dy), y2, x2, weight, mean, rstd, ctx.relu, ctx.has_res and ctx.needs_input_grad[3], _counter(x2),
                    prep(dy2) if dy2 is not None else None)
    dx = _from_2d(out[0], ctx.shape)
    dres = _from_2d(out[3], ctx.shape).to(ctx.res_dtype) if len(out) > 3 else None
    return dx, out[1].to(weight.dtype), out[2].to(weight.dtype), dres


class _BatchNormApply(torch.autograd.Function):
    """Training BatchNorm whose batch statistics were computed elsewhere -- the
    statistics epilogue of the producing convolution (``gemm_core.h`` BnEpi),
    which also updated the running statistics: only the apply pass runs here.
    Backward is the fused BN backward of :class:`_BatchNormAct`."""

    @staticmethod
    def forward(ctx, x, weight, bias, residual, mean, rstd, coef, relu, fork=False):
        shape = x.shape
        x2 = _nhwc_2d(x)
        r2 = _nhwc_2d(residual.to(x.dtype)) if residual is not None else None
        y2 = _bx().apply_train(x2, r2, coef, bool(relu))
        ctx.save_for_backward(x2, y2, weight, mean, rstd)
        ctx.shape, ctx.relu, ctx.has_res = shape, bool(relu), residual is not None
        ctx.res_dtype = residual.dtype if residual is not None else None
        return _outputs(ctx, y2, shape, fork)

    @staticmethod
    def backward(ctx, dy, dy2=None):
        return _bn_backward(ctx, *_grads(dy, dy2)) + (None,) * 5


def batch_norm_apply(x: torch.Tensor, bn: nn.BatchNorm2d, mean: torch.Tensor, rstd: torch.Tensor, coef: torch.Tensor,
                     residual: Optional[torch.Tensor] = None, relu: bool = True, fork: bool = False):
    """``act(bn(x) [+ residual])`` in training mode with precomputed statistics (see :class:`_BatchNormApply`);
    ``fork``: a pair of outputs (see :func:`batch_norm_act`)."""
    return _BatchNormApply.apply(x, bn.weight, bn.bias, residual, mean, rstd, coef, relu, bool(fork))


def fused_stats_ok(bn: nn.BatchNorm2d) -> bool:
    """A training BatchNorm whose statistics a producing kernel can compute (see ops.conv.conv_bn_act)."""
    return (bn.training and bn.momentum is not None and bn.affine and bn.weight.dtype == torch.float32
            and bn.bias.dtype == torch.float32 and bn.weight.is_contiguous() and bn.bias.is_contiguous())


def _native_ok(x: torch.Tensor, bn: nn.BatchNorm2d, residual: Optional[torch.Tensor]) -> bool:
    from p2pfl_amd.ops import _gpu

    if not (_gpu(x) and x.dim() == 4 and x.dtype in (torch.bfloat16, torch.float32)):
        return False
    if not x.is_contiguous(memory_format=torch.channels_last) or x.shape[1] % 8 or x.numel() == 0:
        return False
    if not bn.affine or bn.weight.dtype != torch.float32 or bn.bias.dtype != torch.float32:
        return False
    if residual is not None and (residual.shape != x.shape or not residual.is_contiguous(memory_format=torch.channels_last)):
        return False
    # 16-byte aligned rows of 8 channels
    return x.data_ptr() % 16 == 0 and (residual is None or residual.data_ptr() % 16 == 0)


def batch_norm_act(x: torch.Tensor, bn: nn.BatchNorm2d, residual: Optional[torch.Tensor] = None, relu: bool = True,
                   fork: bool = False):
    """``act(bn(x) [+ residual])`` for a ``BatchNorm2d`` module, fused on MI355X.

    ``fork=True`` returns a pair ``(y, y_alias)`` for an output with two consumers (a
    residual block's first convolution and its shortcut): on the fused training path
    the two branches' gradients reach this BN's backward kernels separately and are
    summed there, so autograd runs no add pass for them.  Elsewhere the pair is
    ``(y, y)``."""
    if fork:
        if _native_ok(x, bn, residual) and (bn.training or not bn.track_running_stats) and bn.momentum is not None:
            track = bn.training and bn.track_running_stats
            rm = bn.running_mean if track else None
            rv = bn.running_var if track else None
            nbt = bn.num_batches_tracked if track and bn.num_batches_tracked is not None else None
            return _BatchNormAct.apply(x, bn.weight, bn.bias, residual, rm, rv, nbt, bn.momentum, bn.eps, relu, True)
        y = batch_norm_act(x, bn, residual, relu)
        return y, y
    training = bn.training or not bn.track_running_stats
    if not _native_ok(x, bn, residual) or (training and bn.momentum is None):
        y = bn(x)
        if residual is not None:
            y = y + residual
        return torch.relu(y) if relu else y
    if training:
        track = bn.training and bn.track_running_stats
        rm = bn.running_mean if track else None
        rv = bn.running_var if track else None
        nbt = bn.num_batches_tracked if track and bn.num_batches_tracked is not None else None
        return _BatchNormAct.apply(x, bn.weight, bn.bias, residual, rm, rv, nbt, bn.momentum, bn.eps, relu)
    if torch.is_grad_enabled() and (x.requires_grad or bn.weight.requires_grad):
        # eval-mode BN with autograd (rare): PyTorch chain
        return batch_norm_act_reference(x, bn.weight, bn.bias, bn.running_mean, bn.running_var, False, 0.0, bn.eps, residual, relu)
    if any(t.data_ptr() % 16 for t in (bn.weight, bn.bias, bn.running_mean, bn.running_var)):
        return batch_norm_act_reference(x, bn.weight, bn.bias, bn.running_mean, bn.running_var, False, 0.0, bn.eps, residual, relu)
    r2 = _nhwc_2d(residual.to(x.dtype)) if residual is not None else None
    y2 = _bx().fwd_eval(_nhwc_2d(x), bn.weight, bn.bias, r2, bn.running_mean, bn.running_var, float(bn.eps), bool(relu))
    return _from_2d(y2, x.shape)
