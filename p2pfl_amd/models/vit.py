"""Vision Transformer (ViT-B/16 for BASELINE.json config 4; small variants for tests).

Not in the reference (SURVEY §7.2 target architecture).  Pre-norm encoder
(Dosovitskiy et al.): 16x16 patch embedding, class token, learned position
embedding, ``depth`` blocks of LayerNorm -> multi-head self-attention ->
residual -> LayerNorm -> MLP(GELU) -> residual, final LayerNorm and a linear
head.  ViT-B/16 at 224x224: 197 tokens, width 768, 12 heads, 12 layers,
MLP 3072, 86.6 M parameters.

On an AMD GPU with the native extension loaded, the fused ops come from
:mod:`p2pfl_amd.ops` (hand-written HIP kernels): LayerNorm forward/backward,
bias+GELU forward/backward and the softmax cross-entropy loss; every Linear
product (patch embedding, QKV, projection, MLP, head -- forward, input and
weight gradient) is the hand-written MFMA GEMM of ``csrc/gemm_pp.hip`` /
``csrc/gemm.hip`` (``ops.linear``: per-shape kernel configuration, bias / GELU /
pre-activation in the epilogue) and multi-head attention is the hand-written
MFMA kernel of ``csrc/attention.hip`` (forward + two-pass backward, straight on
the QKV projection layout).  Optimiser: AdamW (fused over the arena by the learner).
"""

from __future__ import annotations

import math
import os
from typing import Optional

import torch
from torch import nn

from p2pfl_amd import ops
from p2pfl_amd.models.base import FLModule, seed_everything


def _fused(x: torch.Tensor) -> bool:
    return x.is_cuda and ops.available()


# The classifier reads only the class token of the last block's output, and every op
# after that block's attention (projection, residual adds, LayerNorms, MLP) is per
# token: the fused encoder runs them on the B class-token rows alone.  The output and
# every gradient are the same function of the inputs (the other rows' outputs of those
# ops are never read, and their gradients are exactly zero); the attention itself still
# runs over all tokens.  P2PFL_VIT_CLS_ONLY=0 computes the dead rows too.
_CLS_ONLY = os.environ.get("P2PFL_VIT_CLS_ONLY", "1") != "0"


class LayerNorm(nn.LayerNorm):
    """nn.LayerNorm whose GPU path is the fused HIP kernel."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if _fused(x):
            return ops.layer_norm(x, self.weight, self.bias, self.eps)
        return super().forward(x)


class Mlp(nn.Module):
    def __init__(self, dim: int, hidden: int) -> None:
        super().__init__()
        self.fc1 = nn.Linear(dim, hidden)
        self.fc2 = nn.Linear(hidden, dim)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if _fused(x):
            h = ops.linear_gelu(x, self.fc1.weight, self.fc1.bias)  # bias + GELU in the GEMM epilogue
            return ops.linear(h, self.fc2.weight, self.fc2.bias)
        return self.fc2(nn.functional.gelu(self.fc1(x)))


class Attention(nn.Module):
    def __init__(self, dim: int, heads: int) -> None:
        super().__init__()
        self.heads = heads
        self.qkv = nn.Linear(dim, dim * 3)
        self.proj = nn.Linear(dim, dim)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        B, T, C = x.shape
        if _fused(x):
            # HIP kernel on the [B, T, 3C] projection: no head permute / transpose copies
            qkv = ops.linear(x, self.qkv.weight, self.qkv.bias)
            return ops.linear(ops.attention_qkv(qkv, self.heads), self.proj.weight, self.proj.bias)
        qkv = self.qkv(x).view(B, T, 3, self.heads, C // self.heads).permute(2, 0, 3, 1, 4)
        y = nn.functional.scaled_dot_product_attention(qkv[0], qkv[1], qkv[2])
        return self.proj(y.transpose(1, 2).reshape(B, T, C))

    def forward_cls(self, x: torch.Tensor) -> torch.Tensor:
        """``forward(x)[:, 0]`` ([B, C]): attention over every token, the projection of
        the class-token rows only (a strided row view, read in place by the GEMM)."""
        if _fused(x):
            qkv = ops.linear(x, self.qkv.weight, self.qkv.bias)
            return ops.linear(ops.attention_qkv(qkv, self.heads)[:, 0], self.proj.weight, self.proj.bias)
        return self.forward(x)[:, 0]


class Block(nn.Module):
    def __init__(self, dim: int, heads: int, mlp_ratio: float) -> None:
        super().__init__()
        self.norm1 = LayerNorm(dim, eps=1e-6)
        self.attn = Attention(dim, heads)
        self.norm2 = LayerNorm(dim, eps=1e-6)
        self.mlp = Mlp(dim, int(dim * mlp_ratio))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = x + self.attn(self.norm1(x))
        return x + self.mlp(self.norm2(x))


class ViT(FLModule):
    takes_uint8 = True  # forward folds the /255 of a uint8 batch into its first kernel

    def __init__(
        self,
        img_size: int = 224,
        patch: int = 16,
        in_channels: int = 3,
        num_classes: int = 1000,
        dim: int = 768,
        depth: int = 12,
        heads: int = 12,
        mlp_ratio: float = 4.0,
        lr_rate: float = 3e-4,
        weight_decay: float = 0.05,
        seed: Optional[int] = None,
    ) -> None:
        super().__init__()
        if seed is not None:
            seed_everything(seed)
        self.lr_rate, self.weight_decay = lr_rate, weight_decay
        self.patch_embed = nn.Conv2d(in_channels, dim, patch, patch)
        n = (img_size // patch) ** 2
        self.cls_token = nn.Parameter(torch.zeros(1, 1, dim))
        self.pos_embed = nn.Parameter(torch.zeros(1, n + 1, dim))
        self.blocks = nn.Sequential(*[Block(dim, heads, mlp_ratio) for _ in range(depth)])
        self.norm = LayerNorm(dim, eps=1e-6)
        self.head = nn.Linear(dim, num_classes)
        nn.init.trunc_normal_(self.pos_embed, std=0.02)
        nn.init.trunc_normal_(self.cls_token, std=0.02)
        for m in self.modules():
            if isinstance(m, nn.Linear):
                nn.init.trunc_normal_(m.weight, std=0.02)
                nn.init.zeros_(m.bias)
        w = self.patch_embed.weight
        nn.init.uniform_(w, -1 / math.sqrt(w[0].numel()), 1 / math.sqrt(w[0].numel()))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        P = self.patch_embed.weight.shape[-1]
        if x.dtype == torch.uint8 and _fused(x) and P % 8 == 0 and x.shape[2] % P == 0 and x.shape[3] % P == 0:
            # one kernel: uint8 -> bf16 patch rows / 255 (the same values the float cast, the
            # scale and the GEMM's bf16 cast produced), then the patch-embedding GEMM
            w = self.patch_embed.weight
            x = ops.linear(ops.patchify_u8(x, P), w.view(w.shape[0], -1), self.patch_embed.bias)
        else:
            if x.dtype == torch.uint8:
                x = x.float().mul_(1.0 / 255.0)
            x = self._patchify_embed(x)
        # class token + position embedding (one kernel each way on the GPU, bf16)
        x = ops.embed_tokens(x, self.cls_token, self.pos_embed) if _fused(x) else (
            torch.cat([self.cls_token.expand(x.shape[0], -1, -1).to(x.dtype), x], dim=1) + self.pos_embed.to(x.dtype))
        if _fused(x):
            y = self._encoder_fused(x)
            return ops.linear(y if y.dim() == 2 else y[:, 0], self.head.weight, self.head.bias)
        x = self.norm(self.blocks(x))
        return self.head(x[:, 0])

    def _encoder_fused(self, h: torch.Tensor) -> torch.Tensor:
        """The block stack with every residual add fused into the following LayerNorm.

        ``h`` is the residual stream; ``add_layer_norm`` returns the new stream
        and its normalisation (norm2 of the same block, or norm1 of the next /
        the final norm), so no separate add kernel runs forward or backward.
        With ``_CLS_ONLY`` the last block continues from its attention on the
        class-token rows only and the result is [B, C] (else [B, T, C]).
        """
        blocks = list(self.blocks)
        y = blocks[0].norm1(h)
        for i, blk in enumerate(blocks):
            if _CLS_ONLY and i + 1 == len(blocks):
                h0, y0 = ops.add_layer_norm(h[:, 0], blk.attn.forward_cls(y), blk.norm2.weight, blk.norm2.bias,
                                            blk.norm2.eps)
                return ops.add_layer_norm(h0, blk.mlp(y0), self.norm.weight, self.norm.bias, self.norm.eps)[1]
            h, y = ops.add_layer_norm(h, blk.attn(y), blk.norm2.weight, blk.norm2.bias, blk.norm2.eps)
            nxt = blocks[i + 1].norm1 if i + 1 < len(blocks) else self.norm
            h, y = ops.add_layer_norm(h, blk.mlp(y), nxt.weight, nxt.bias, nxt.eps)
        return y

    def _patchify_embed(self, x: torch.Tensor) -> torch.Tensor:
        """Conv2d(C, D, P, stride=P) as patchify + one GEMM (identical math).

        MIOpen has no tuned solver for the 16x16 / stride-16 convolution and
        falls back to its naive kernel (measured 2.8 ms per call on MI355X at
        batch 32); as [B*196, C*P*P] x [C*P*P, D] it is a plain hipBLASLt GEMM.
        The conv weight [D, C, P, P] flattens in exactly the patch order.
        """
        w = self.patch_embed.weight
        D, C, P, _ = w.shape
        B, _, H, W = x.shape
        patches = x.view(B, C, H // P, P, W // P, P).permute(0, 2, 4, 1, 3, 5).reshape(B, (H // P) * (W // P), C * P * P)
        if _fused(patches):
            return ops.linear(patches, w.view(D, C * P * P), self.patch_embed.bias)
        return nn.functional.linear(patches, w.view(D, C * P * P), self.patch_embed.bias)

    def loss_fn(self, out: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
        if _fused(out):
            return ops.softmax_xent(out, y)
        return nn.functional.cross_entropy(out, y)

    def fp32_parameter_names(self) -> set:
        """Parameters the fused kernels read in fp32 (LayerNorm affine, the bias of bias+GELU).

        Every other weight (GEMM matrices, plain-linear biases, tokens) is a bf16
        view of the learner's shadow arena under mixed precision.
        """
        return {n for n, _ in self.named_parameters() if "norm" in n or n.endswith("fc1.bias")}

    def configure_optimizers(self) -> torch.optim.Optimizer:
        return torch.optim.AdamW(self.parameters(), lr=self.lr_rate, weight_decay=self.weight_decay)


def ViT_B16(num_classes: int = 1000, img_size: int = 224, **kw) -> ViT:
    return ViT(img_size=img_size, patch=16, num_classes=num_classes, dim=768, depth=12, heads=12, **kw)


def ViT_Tiny(num_classes: int = 10, img_size: int = 32, patch: int = 4, **kw) -> ViT:
    """Small test variant (CIFAR-sized input)."""
    return ViT(img_size=img_size, patch=patch, num_classes=num_classes, dim=192, depth=4, heads=3, **kw)
