"""Autograd wrappers of the fused transformer / classifier kernels (``csrc/fused_ops.hip``).

``layer_norm``, ``bias_gelu`` and ``softmax_xent`` run the hand-written HIP
kernels for GPU tensors (bf16 or fp32 activations, fp32 parameters) and plain
PyTorch otherwise; the ``*_reference`` functions are the fp32 PyTorch
definitions the numerics tests compare against.
"""

from __future__ import annotations

import os
import threading
from contextlib import contextmanager

import torch
import torch.nn.functional as F


def _native(x: torch.Tensor) -> bool:
    from p2pfl_amd.ops import _gpu

    return _gpu(x) and x.dtype in (torch.bfloat16, torch.float32)


def _fx():
    from p2pfl_amd.ops import ext

    return ext().fused


# -- references ---------------------------------------------------------------
def layer_norm_reference(x, w, b, eps):
    return F.layer_norm(x.float(), (x.shape[-1],), w.float(), b.float(), eps)


def bias_gelu_reference(x, b):
    return F.gelu(x.float() + b.float())


def softmax_xent_reference(z, y):
    return F.cross_entropy(z.float(), y)


def attention_qkv_reference(qkv, heads):
    """fp32 multi-head self-attention over a [B, T, 3C] QKV projection -> [B, T, C]."""
    B, T, C3 = qkv.shape
    C = C3 // 3
    q, k, v = qkv.float().view(B, T, 3, heads, C // heads).permute(2, 0, 3, 1, 4)
    y = F.scaled_dot_product_attention(q, k, v)
    return y.transpose(1, 2).reshape(B, T, C)


# -- deferred parameter-gradient reductions ------------------------------------------
# A parameter gradient that is a column sum over the batch rows (LayerNorm dgamma /
# dbeta, a linear bias gradient, the bias gradient of the fused GELU backward) is a
# [S, C] partial-sum pass followed by a small fixed-order reduction launch (~5 us,
# latency-bound): 73 of them per ViT-B/16 step.  Inside ``deferred_param_grads()``
# (the training step graphs' backward) the backward passes return their partials
# instead; on exit ONE ``col_reduce_multi`` launch reduces them all -- bitwise the
# same sums -- and assigns the parameters' ``.grad`` (the autograd output for those
# parameters is None).  The context must enclose the FORWARD too: a Function records
# the open collection in its ctx when it runs forward (on the caller's thread), since
# autograd runs CUDA backward nodes on its own device thread -- so another peer's
# concurrent backward can never land in this step's collection.
# P2PFL_DEFER_GRAD_REDUCE=0 keeps the per-pass reductions.
_DEFER_ON = os.environ.get("P2PFL_DEFER_GRAD_REDUCE", "1") != "0"
# the bias column sums themselves too (their partial pass batched as well); P2PFL_DEFER_COLSUM=0:
# partials per backward pass, only the reductions batched
_DEFER_COLSUM = os.environ.get("P2PFL_DEFER_COLSUM", "1") != "0"
_TLS = threading.local()


class _Deferred:
    def __init__(self) -> None:
        self.open = True
        self.params: list = []
        self.parts: list = []
        self.cs_params: list = []  # bias gradients = column sums of activations, partials deferred too
        self.cs_x: list = []


def defer_scope():
    """The collection a Function's forward should record in its ctx (None outside one)."""
    return getattr(_TLS, "d", None)


def defer_grad(d, param, part: torch.Tensor) -> bool:
    """Register ``param``'s gradient as the column sums of ``part`` ([S, C] fp32) in the
    collection ``d`` recorded at forward time; False (reduce now) if there is none."""
    if d is None or not d.open or not isinstance(param, torch.nn.Parameter):
        return False
    d.params.append(param)
    d.parts.append(part)
    return True


def defer_colsum(d, param, x: torch.Tensor) -> bool:
    """Register ``param``'s gradient as the column sums of the bf16 activation ``x``
    ([N, H], kept alive until the exit): both the partial pass and the reduction run
    batched at the exit.  False (reduce now) without an open collection."""
    if (not _DEFER_COLSUM or d is None or not d.open or not isinstance(param, torch.nn.Parameter) or x.dtype != torch.bfloat16
            or x.dim() != 2 or not x.is_contiguous() or x.shape[0] == 0 or x.shape[1] % 8 or x.data_ptr() % 16):
        return False
    d.cs_params.append(param)
    d.cs_x.append(x)
    return True


@contextmanager
def deferred_param_grads(enabled: bool = True):
    """Wrap the forward AND backward of a training step: the deferrable parameter-gradient
    reductions of its backward run as one launch on exit, which also sets ``.grad``."""
    if not (enabled and _DEFER_ON) or getattr(_TLS, "d", None) is not None:
        yield
        return
    d = _TLS.d = _Deferred()
    try:
        yield
    finally:
        _TLS.d = None
        d.open = False
    if d.cs_x:  # the bias partials of every deferred column sum: one launch
        fx = _fx()
        parts = [torch.empty(fx.colsum_splits(x.shape[0]), x.shape[1], dtype=torch.float32, device=x.device)
                 for x in d.cs_x]
        fx.column_sum_parts_multi(d.cs_x, parts)
        d.params += d.cs_params
        d.parts += parts
        d.cs_x.clear()
    if not d.parts:
        return
    outs = [torch.empty(p.shape, dtype=p.dtype, device=part.device) for p, part in zip(d.params, d.parts)]
    _fx().col_reduce_multi(d.parts, [o.view(-1) for o in outs])
    for p, g in zip(d.params, outs):
        if p.grad is None:
            p.grad = g
        else:
            p.grad.add_(g)


# -- LayerNorm ----------------------------------------------------------------
def _ln_bwd(ctx, dy2, x2, w, mean, rstd, gs2=None):
    """dx, dgamma, dbeta -- the parameter gradients deferred where possible (None)."""
    wp, bp = ctx.params
    d = ctx.defer
    if d is not None and d.open and (ctx.needs_input_grad[ctx.wi] or ctx.needs_input_grad[ctx.wi + 1]):
        dx, pdw, pdb = _fx().ln_bwd_parts(dy2, x2, w.contiguous(), mean, rstd, gs2)
        dw = None if ctx.needs_input_grad[ctx.wi] and defer_grad(d, wp, pdw) else pdw.sum(0).to(w.dtype)
        db = None if ctx.needs_input_grad[ctx.wi + 1] and defer_grad(d, bp, pdb) else pdb.sum(0).to(w.dtype)
        return dx, dw, db
    dx, dw, db = _fx().ln_bwd(dy2, x2, w.contiguous(), mean, rstd, gs2)
    return dx, dw.to(w.dtype), db.to(w.dtype)


class _LayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, eps):
        shape = x.shape
        x2 = x.reshape(-1, shape[-1]).contiguous()
        y, mean, rstd = _fx().ln_fwd(x2, w.contiguous(), b.contiguous(), float(eps))
        ctx.save_for_backward(x2, w, mean, rstd)
        ctx.shape = shape
        ctx.params, ctx.wi, ctx.defer = (w, b), 1, defer_scope()
        return y.view(shape)

    @staticmethod
    def backward(ctx, dy):
        x2, w, mean, rstd = ctx.saved_tensors
        dy2 = dy.reshape(x2.shape).to(x2.dtype).contiguous()
        dx, dw, db = _ln_bwd(ctx, dy2, x2, w, mean, rstd)
        return dx.view(ctx.shape), dw, db, None


def layer_norm(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor, eps: float = 1e-5) -> torch.Tensor:
    """LayerNorm over the last dim; output dtype = input dtype (statistics in fp32)."""
    C = x.shape[-1]
    if (
        _native(x)
        and weight is not None
        and bias is not None
        and weight.dtype == torch.float32
        and C % 8 == 0
        and C <= 2048
    ):
        return _LayerNorm.apply(x, weight, bias, eps)
    return F.layer_norm(x, (C,), weight, bias, eps)


# -- residual add + LayerNorm -----------------------------------------------------
class _AddLayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, r, w, b, eps):
        shape = x.shape
        x2 = x.reshape(-1, shape[-1]).contiguous()
        r2 = r.reshape(x2.shape).to(x2.dtype).contiguous()
        y, mean, rstd, s = _fx().ln_fwd(x2, w.contiguous(), b.contiguous(), float(eps), r2)
        ctx.save_for_backward(s, w, mean, rstd)
        ctx.shape = shape
        ctx.params, ctx.wi, ctx.defer = (w, b), 2, defer_scope()
        return s.view(shape), y.view(shape)

    @staticmethod
    def backward(ctx, gs, dy):
        s, w, mean, rstd = ctx.saved_tensors
        if dy is None:
            dy = torch.zeros_like(s)
        dy2 = dy.reshape(s.shape).to(s.dtype).contiguous()
        gs2 = gs.reshape(s.shape).to(s.dtype).contiguous() if gs is not None else None
        dx, dw, db = _ln_bwd(ctx, dy2, s, w, mean, rstd, gs2)
        dx = dx.view(ctx.shape)
        return dx, dx, dw, db, None


def add_layer_norm_reference(x, r, w, b, eps):
    s = (x + r).to(x.dtype)
    return s, F.layer_norm(s.float(), (x.shape[-1],), w.float(), b.float(), eps).to(x.dtype)


def add_layer_norm(x: torch.Tensor, r: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor, eps: float = 1e-5):
    """``s = x + r; return s, LayerNorm(s)`` in one pass (one pass back: dx = dr = ds + LN'(dy))."""
    C = x.shape[-1]
    if _native(x) and r.shape == x.shape and weight.dtype == torch.float32 and C % 8 == 0 and C <= 2048:
        return _AddLayerNorm.apply(x, r, weight, bias, eps)
    s = x + r
    return s, F.layer_norm(s, (C,), weight, bias, eps)


# -- linear with a fused bias gradient -------------------------------------------------
def _wgrad_splits(M: int, N: int, K: int) -> int:
    """Split-K factor for dW[N, K] = dy[M, N]^T x[M, K] (measured on MI355X, tools/lab/wgrad_splitk_bench.py).

    The ViT weight gradients have only 36-144 128x128 output tiles for 256
    CUs but a 6304-long reduction: splitting the reduction into batches of a
    bmm fills the chip (proj 46.9 -> 33.9 us, fc1 69.3 -> 55.0, fc2 68.2 ->
    54.3, qkv 58.6 -> 54.4 with 2 splits).
    """
    if M < 4096:
        return 1
    tiles = -(-N // 128) * -(-K // 128)
    s = 2 if 96 <= tiles < 144 else 4
    while s > 1 and M % s:
        s //= 2
    return s


def _wgrad(dy2: torch.Tensor, x2: torch.Tensor) -> torch.Tensor:
    M, N = dy2.shape
    K = x2.shape[1]
    s = _wgrad_splits(M, N, K)
    if s == 1:
        return torch.mm(dy2.t(), x2)
    part = torch.bmm(dy2.view(s, M // s, N).transpose(1, 2), x2.contiguous().view(s, M // s, K))
    if part.dtype == torch.bfloat16 and (N * K) % 8 == 0:
        return _fx().split_sum_bf16(part)  # one pass, fp32 accumulation, bf16 out
    return part.sum(0, dtype=torch.float32).to(dy2.dtype)



class _Linear(torch.autograd.Function):
    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda", cast_inputs=torch.bfloat16)
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        ctx.has_bias = b is not None
        ctx.bias_dtype = b.dtype if b is not None else None
        return F.linear(x, w, b)

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1])
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = torch.mm(dy2, w).view(*dy.shape[:-1], w.shape[1])
        if ctx.needs_input_grad[1]:
            dw = _wgrad(dy2, x.reshape(-1, x.shape[-1]))
        if ctx.has_bias and ctx.needs_input_grad[2]:
            # one streaming pass, not a generic reduce; a bf16 bias gets its bf16 gradient directly
            db = _fx().column_sum(dy2, ctx.bias_dtype == torch.bfloat16).to(ctx.bias_dtype)
        return dx, dw, db


def linear(x: torch.Tensor, weight: torch.Tensor, bias=None) -> torch.Tensor:
    """``F.linear`` whose backward computes the bias gradient with the column-sum kernel
    and the weight gradient with a split-K batched GEMM at ViT sizes."""
    if _native(x) and weight.shape[0] % 8 == 0:
        return _Linear.apply(x, weight, bias)
    return F.linear(x, weight, bias)


# -- bias + GELU ----------------------------------------------------------------
class _BiasGelu(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, b):
        xc = x.contiguous()
        ctx.save_for_backward(xc, b)
        return _fx().bias_gelu_fwd(xc, b.contiguous())

    @staticmethod
    def backward(ctx, dy):
        x, b = ctx.saved_tensors
        dx, db = _fx().bias_gelu_bwd(dy.to(x.dtype).contiguous(), x, b.contiguous())
        return dx, db.to(b.dtype)


def bias_gelu(x: torch.Tensor, bias: torch.Tensor) -> torch.Tensor:
    """``gelu(x + bias)`` (exact erf GELU) with bias broadcast over the last dim."""
    if _native(x) and bias.dtype == torch.float32 and x.shape[-1] % 8 == 0:
        return _BiasGelu.apply(x, bias)
    return F.gelu(x + bias.to(x.dtype))


# -- softmax cross-entropy --------------------------------------------------------
class _SoftmaxXent(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z, y):
        zc = z.contiguous()
        loss_rows, lse = _fx().xent_fwd(zc, y.contiguous())
        ctx.save_for_backward(zc, y, lse)
        return loss_rows.mean()

    @staticmethod
    def backward(ctx, g):
        z, y, lse = ctx.saved_tensors
        gs = g.detach().float().reshape(1).contiguous()
        return _fx().xent_bwd(z, y, lse, gs), None


def softmax_xent(logits: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
    """Mean softmax cross-entropy (= ``F.cross_entropy`` with integer labels), fp32 result."""
    if _native(logits) and logits.dim() == 2 and labels.dtype == torch.int64 and labels.is_cuda:
        return _SoftmaxXent.apply(logits, labels)
    return F.cross_entropy(logits, labels)


# -- multi-head self-attention --------------------------------------------------------
class _EmbedTokens(torch.autograd.Function):
    """``cat([cls, y], 1) + pos`` of a ViT in one kernel each way (``csrc/fused_ops.hip``
    embed_tokens_*): the backward writes the patch tokens' gradient contiguously for the
    patch-embedding GEMM and the batch sums of the position / class-token gradients."""

    @staticmethod
    def forward(ctx, y, cls, pos):
        ctx.shapes = (cls.shape, pos.shape)
        return _fx().embed_tokens_fwd(y.contiguous(), cls.contiguous().view(-1), pos.contiguous().view(-1, y.shape[-1]))

    @staticmethod
    def backward(ctx, dh):
        dy, dpos, dcls = _fx().embed_tokens_bwd(dh.to(torch.bfloat16).contiguous())
        cs, ps = ctx.shapes
        return dy, dcls.view(cs), dpos.view(ps)


def embed_tokens(y: torch.Tensor, cls: torch.Tensor, pos: torch.Tensor) -> torch.Tensor:
    """``torch.cat([cls.expand(B, -1, -1), y], 1) + pos`` for bf16 ViT tokens on the GPU."""
    if _native(y) and y.dtype == cls.dtype == pos.dtype == torch.bfloat16 and y.shape[-1] % 8 == 0:
        return _EmbedTokens.apply(y, cls, pos)
    return torch.cat([cls.expand(y.shape[0], -1, -1).to(y.dtype), y], dim=1) + pos.to(y.dtype)


def patchify_u8(x: torch.Tensor, patch: int) -> torch.Tensor:
    """uint8 images [B, C, H, W] -> bf16 patch rows [B, (H/P)(W/P), C P P] scaled by 1/255 (one kernel)."""
    return _fx().patchify_u8(x.contiguous(), int(patch))


class _AttentionQKV(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, heads):
        qkv = qkv.contiguous()
        o, lse = _fx().attn_fwd(qkv, int(heads))
        ctx.save_for_backward(qkv, o, lse)
        ctx.heads = int(heads)
        return o

    @staticmethod
    def backward(ctx, do):
        qkv, o, lse = ctx.saved_tensors
        return _fx().attn_bwd(qkv, o, do.to(o.dtype).contiguous(), lse, ctx.heads), None


def attention_qkv(qkv: torch.Tensor, heads: int) -> torch.Tensor:
    """softmax(q k^T / sqrt(d)) v for every head of a [B, T, 3C] QKV projection -> [B, T, C].

    The HIP kernel (head dim 64, T <= 256, bf16) reads q/k/v straight out of
    the projection and writes the proj GEMM's input layout; other shapes use
    PyTorch SDPA.
    """
    B, T, C3 = qkv.shape
    C = C3 // 3
    if _native(qkv) and qkv.dtype == torch.bfloat16 and C == heads * 64 and T <= 256:
        return _AttentionQKV.apply(qkv, heads)
    q, k, v = qkv.view(B, T, 3, heads, C // heads).permute(2, 0, 3, 1, 4)
    return F.scaled_dot_product_attention(q, k, v).transpose(1, 2).reshape(B, T, C)
