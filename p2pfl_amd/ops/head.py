"""Classification head on two HIP launches (``csrc/head.hip``).

``global average pool -> Linear (<= 64 classes) -> softmax cross-entropy``: the
tail of the ResNet family.  :func:`head_xent` returns ``(loss, logits,
accuracy)`` from one forward launch; its backward is one launch producing the
feature-map gradient (bf16, channels-last), ``dW`` and ``db``.  PyTorch-ROCm
runs the same tail as a dozen launches, among them a hipBLASLt GEMM.  The
reference's head: ``nn.Linear`` + ``CrossEntropyLoss``
(``/root/reference/p2pfl/learning/pytorch/mnist_examples/models/cnn.py:71-98``).
"""

from __future__ import annotations

from typing import Optional, Tuple

import torch
from torch import nn


def _C():
    from p2pfl_amd.ops import ext

    return ext()


def head_ok(f: torch.Tensor, fc: nn.Linear, y: Optional[torch.Tensor]) -> bool:
    from p2pfl_amd.ops import _gpu

    if not _gpu(f) or f.dim() != 4 or f.dtype != torch.bfloat16 or not f.is_contiguous(memory_format=torch.channels_last):
        return False
    w, b = fc.weight, fc.bias
    if w.dim() != 2 or w.shape[1] != f.shape[1] or not (1 <= w.shape[0] <= 64) or not w.is_contiguous():
        return False
    if w.dtype not in (torch.float32, torch.bfloat16) or (b is not None and (b.dtype != torch.float32 or not b.is_contiguous())):
        return False
    return y is None or (y.dtype == torch.int64 and y.dim() == 1 and y.shape[0] == f.shape[0])


class _HeadXent(torch.autograd.Function):
    @staticmethod
    def forward(ctx, f, w, b, y):
        from p2pfl_amd.ops import splitk

        f4 = f.permute(0, 2, 3, 1)
        if not f4.is_contiguous() or f4.data_ptr() % 16:
            f4 = f4.contiguous()
        y = y.contiguous()
        pooled, logits, loss, acc = _C().head.fwd(f4, w, b, y, splitk.counters(1, f.device))
        ctx.save_for_backward(logits, y, pooled, w)
        ctx.fshape = list(f4.shape)
        ctx.has_b = b is not None
        ctx.mark_non_differentiable(logits, acc)
        ctx.set_materialize_grads(False)  # no zero-filled gradients for logits / accuracy
        return loss, logits, acc

    @staticmethod
    def backward(ctx, gloss, _glogits, _gacc):
        logits, y, pooled, w = ctx.saved_tensors
        df4, dw, db = _C().head.bwd(gloss.float().reshape(1), logits, y, pooled, w, ctx.fshape)
        return df4.permute(0, 3, 1, 2), dw, (db if ctx.has_b else None), None


def head_xent(f: torch.Tensor, fc: nn.Linear, y: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """``(mean cross-entropy, logits, accuracy)`` of ``fc(avgpool(f))`` against ``y`` (:func:`head_ok`)."""
    return _HeadXent.apply(f, fc.weight, fc.bias, y)


def head_reference(f: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor], y: torch.Tensor):
    """fp32 definition used by the numerics tests."""
    p = f.float().mean(dim=(2, 3))
    logits = p @ w.float().t() + (b.float() if b is not None else 0.0)
    return nn.functional.cross_entropy(logits, y), logits
