"""ResNet-18/34/50 (BASELINE.json configs 3 and 5).

Not in the reference (its zoo is the MNIST MLP/CNN only);
these are the target architectures of the MI355X build plan.
Standard He et al. layouts; ``stem="cifar"`` uses the 3x3/stride-1 stem
without max-pool for 32x32 inputs, ``stem="imagenet"`` the 7x7/stride-2 stem
plus max-pool.  Inputs are uint8 images (the data modules keep datasets as
uint8 on the device); normalisation to [0, 1] happens in ``forward``.

Activations run channels-last on the GPU.  What runs per convolution
(:func:`~p2pfl_amd.ops.conv.conv2d`):

* 1x1 convolutions (bottlenecks, downsample shortcuts) run on the same
  implicit-GEMM conv kernels as the 3x3 ones, tuned per shape by the eager step
  (``P2PFL_CONV1X1_MODE=gemm``: as native GEMMs over the channels-last pixels,
  :func:`~p2pfl_amd.ops.conv.conv1x1_gemm` -> :func:`~p2pfl_amd.ops.gemm.linear`);
* every other convolution but the 3-channel stem, inside the captured HIP step
  graphs (all full-batch training and evaluation steps), runs on the
  hand-written implicit-GEMM MFMA kernels (``csrc/conv.hip``: forward, input and
  weight gradient, reading the learner's channels-last bf16 weight shadow) --
  MIOpen convolutions replayed from graphs were not memory-safe
  (``profiles/r3_nan_root_cause.md``); eager steps (short last batches) take
  whichever of the native kernels and MIOpen measured faster;
* the 3-channel stem runs the direct small-C kernels of ``csrc/stem.hip``
  (forward + weight gradient, reading the uint8 / fp32 batch as it comes).

In training, BatchNorm runs the separate statistics / finalize / apply kernels of
``csrc/batchnorm.hip`` by default.  With ``P2PFL_CONV_BN_STATS=1`` every convolution's
launch also computes the batch statistics of the BatchNorm that follows it
(``gemm_core.h`` BnEpi) and the input-gradient launch of a block's inner convolution
the backward statistics of the one before it (:func:`~p2pfl_amd.ops.conv.bn_act_conv_bn_stats`):
conv1 -> [bn1 apply, conv2] -> bn2 apply per BasicBlock -- fewer launches, but measured
slower on these shapes (``profiles/r4_bn_epilogue.md``).  Evaluation (running statistics) runs the one-pass
BN kernel of ``csrc/batchnorm.hip`` (:func:`~p2pfl_amd.ops.batchnorm.batch_norm_act`).  Optimiser: SGD with momentum 0.9 and weight decay 5e-4 (fused
into one arena kernel by the learner), a standard federated CIFAR setup.
"""

from __future__ import annotations

import os
from typing import List, Optional, Type, Union

import torch
from torch import nn

from p2pfl_amd.models.base import FLModule, seed_everything
from p2pfl_amd.ops.batchnorm import batch_norm_act, batch_norm_apply
from p2pfl_amd.ops.head import head_ok, head_xent
from p2pfl_amd.ops.conv import bn_act_conv_bn_stats, conv2d, conv_bn_act, conv_bn_stats, stem_conv2d, stem_ok

# NHWC activations on the GPU (P2PFL_CHANNELS_LAST=0 keeps NCHW)
_CHANNELS_LAST = os.environ.get("P2PFL_CHANNELS_LAST", "1") != "0"
# 3-channel stem on the direct HIP kernels (csrc/stem.hip); P2PFL_NATIVE_STEM=0 restores F.conv2d
_NATIVE_STEM = os.environ.get("P2PFL_NATIVE_STEM", "1") != "0"
# pool + fc + cross-entropy on csrc/head.hip (P2PFL_NATIVE_HEAD=0: PyTorch / hipBLASLt)
_NATIVE_HEAD = os.environ.get("P2PFL_NATIVE_HEAD", "1") != "0"


# A block's input feeds its first convolution and its shortcut.  The producing BN
# returns two autograd outputs for them (batch_norm_act(..., fork=True)), so the
# two gradients are summed inside that BN's backward kernels rather than by an
# autograd add pass per block (P2PFL_RESNET_FORK=0: one output, autograd adds).
_FORK = os.environ.get("P2PFL_RESNET_FORK", "1") != "0"


def _pair(x):
    """(input of the first convolution, input of the shortcut) of a block."""
    return x if isinstance(x, tuple) else (x, x)


def _shortcut(sc: nn.Module, x: torch.Tensor) -> torch.Tensor:
    """Identity, or the projection conv + BN (no activation)."""
    if isinstance(sc, nn.Identity):
        return x
    return conv_bn_act(x, sc[0], sc[1], relu=False)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, cin: int, cout: int, stride: int = 1) -> None:
        super().__init__()
        self.conv1 = nn.Conv2d(cin, cout, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(cout)
        self.conv2 = nn.Conv2d(cout, cout, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(cout)
        self.shortcut: nn.Module = nn.Identity()
        if stride != 1 or cin != cout:
            self.shortcut = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))

    def forward(self, x):
        """``x``: a tensor or the (conv input, shortcut input) pair of a forked BN output;
        returns such a pair (see ``_FORK``)."""
        x, xs = _pair(x)
        st = conv_bn_stats(x, self.conv1, self.bn1)
        st = bn_act_conv_bn_stats(st, self.bn1, True, self.conv2, self.bn2) if st is not None else None
        if st is not None:  # conv1 -> [bn1 apply, conv2] -> bn2 apply: 3 launches forward
            return batch_norm_apply(st[0], self.bn2, st[1], st[2], st[3], _shortcut(self.shortcut, xs), True, _FORK)
        out = conv_bn_act(x, self.conv1, self.bn1)
        return conv_bn_act(out, self.conv2, self.bn2, residual=_shortcut(self.shortcut, xs), fork=_FORK)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin: int, width: int, stride: int = 1) -> None:
        super().__init__()
        cout = width * self.expansion
        self.conv1 = nn.Conv2d(cin, width, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = nn.Conv2d(width, width, 3, stride, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = nn.Conv2d(width, cout, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(cout)
        self.shortcut: nn.Module = nn.Identity()
        if stride != 1 or cin != cout:
            self.shortcut = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))

    def forward(self, x):
        """As :meth:`BasicBlock.forward`: a tensor or a pair in, a pair out."""
        x, xs = _pair(x)
        st = conv_bn_stats(x, self.conv1, self.bn1)
        st = bn_act_conv_bn_stats(st, self.bn1, True, self.conv2, self.bn2) if st is not None else None
        st = bn_act_conv_bn_stats(st, self.bn2, True, self.conv3, self.bn3) if st is not None else None
        if st is not None:
            return batch_norm_apply(st[0], self.bn3, st[1], st[2], st[3], _shortcut(self.shortcut, xs), True, _FORK)
        out = conv_bn_act(x, self.conv1, self.bn1)
        out = conv_bn_act(out, self.conv2, self.bn2)
        return conv_bn_act(out, self.conv3, self.bn3, residual=_shortcut(self.shortcut, xs), fork=_FORK)


class ResNet(FLModule):
    takes_uint8 = True  # forward folds the /255 of a uint8 batch into its first kernel

    def __init__(
        self,
        block: Type[Union[BasicBlock, Bottleneck]],
        layers: List[int],
        num_classes: int = 10,
        in_channels: int = 3,
        stem: str = "cifar",
        lr_rate: float = 0.05,
        momentum: float = 0.9,
        weight_decay: float = 5e-4,
        seed: Optional[int] = None,
    ) -> None:
        super().__init__()
        if seed is not None:
            seed_everything(seed)
        self.lr_rate, self.momentum, self.weight_decay = lr_rate, momentum, weight_decay
        if stem == "cifar":
            self.stem = nn.Sequential(nn.Conv2d(in_channels, 64, 3, 1, 1, bias=False), nn.BatchNorm2d(64), nn.ReLU(inplace=True))
        elif stem == "imagenet":
            self.stem = nn.Sequential(
                nn.Conv2d(in_channels, 64, 7, 2, 3, bias=False),
                nn.BatchNorm2d(64),
                nn.ReLU(inplace=True),
                nn.MaxPool2d(3, 2, 1),
            )
        else:
            raise ValueError(f"unknown stem {stem!r}")
        cin = 64
        stages = []
        for i, (n, width) in enumerate(zip(layers, (64, 128, 256, 512))):
            blocks = []
            for j in range(n):
                stride = 2 if (i > 0 and j == 0) else 1
                blocks.append(block(cin, width, stride))
                cin = width * block.expansion
            stages.append(nn.Sequential(*blocks))
        self.layer1, self.layer2, self.layer3, self.layer4 = stages
        self.fc = nn.Linear(cin, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)

    def features(self, x: torch.Tensor) -> torch.Tensor:
        """The last stage's feature map (channels-last on the GPU)."""
        stem = self.stem[0]
        if _NATIVE_STEM and stem_ok(x, stem):
            # direct small-C kernel: reads the batch as it is (uint8 with the 1/255 folded
            # in, or fp32, NCHW) -- no normalisation pass, no channels-last copy, no MIOpen
            x = stem_conv2d(x, stem, 1.0 / 255.0 if x.dtype == torch.uint8 else 1.0)
        else:
            if x.dtype == torch.uint8:
                x = x.float().mul_(1.0 / 255.0)
            if x.is_cuda and _CHANNELS_LAST:
                x = x.contiguous(memory_format=torch.channels_last)
            x = conv2d(x, stem)
        if len(self.stem) > 3:
            x = self.stem[3](batch_norm_act(x, self.stem[1]))
        else:
            x = batch_norm_act(x, self.stem[1], fork=_FORK)
        return _pair(self.layer4(self.layer3(self.layer2(self.layer1(x)))))[0]

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = torch.flatten(nn.functional.adaptive_avg_pool2d(self.features(x), 1), 1)
        return self.fc(x)

    # pool + fc + cross-entropy as two HIP launches (ops/head.py) when the shapes allow
    def _native_head(self, f: torch.Tensor, y: torch.Tensor) -> bool:
        """The fused head computes the default cross-entropy: not for a subclass
        that overrides ``loss_fn``."""
        return _NATIVE_HEAD and type(self).loss_fn is FLModule.loss_fn and head_ok(f, self.fc, y)

    def training_step(self, batch, batch_idx: int) -> torch.Tensor:
        x, y = batch
        f = self.features(x)
        if self._native_head(f, y):
            loss, _, _ = head_xent(f, self.fc, y)
        else:
            loss = self.loss_fn(self.fc(torch.flatten(nn.functional.adaptive_avg_pool2d(f, 1), 1)), y)
        self.log("train_loss", loss, prog_bar=True)
        return loss

    def _eval_step(self, batch, prefix: str) -> torch.Tensor:
        x, y = batch
        f = self.features(x)
        if self._native_head(f, y):
            loss, _, acc = head_xent(f, self.fc, y)
            self.log(f"{prefix}_loss", loss, prog_bar=True)
            self.log(f"{prefix}_metric", acc, prog_bar=True)
            return loss
        return super()._eval_step(batch, prefix)

    def channels_last_parameter_names(self) -> List[str]:
        """Spatial conv weights a mixed-precision arena keeps in channels-last order (NHWC activations)."""
        if not _CHANNELS_LAST:
            return []
        return [n for n, p in self.named_parameters() if p.dim() == 4 and p.shape[2] * p.shape[3] > 1]

    def configure_optimizers(self) -> torch.optim.Optimizer:
        return torch.optim.SGD(self.parameters(), lr=self.lr_rate, momentum=self.momentum, weight_decay=self.weight_decay)


def ResNet18(num_classes: int = 10, stem: str = "cifar", **kw) -> ResNet:
    return ResNet(BasicBlock, [2, 2, 2, 2], num_classes, stem=stem, **kw)


def ResNet34(num_classes: int = 10, stem: str = "cifar", **kw) -> ResNet:
    return ResNet(BasicBlock, [3, 4, 6, 3], num_classes, stem=stem, **kw)


def ResNet50(num_classes: int = 10, stem: str = "cifar", **kw) -> ResNet:
    return ResNet(Bottleneck, [3, 4, 6, 3], num_classes, stem=stem, **kw)
