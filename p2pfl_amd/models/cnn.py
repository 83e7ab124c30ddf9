"""MNIST LeNet-style CNN (reference ``mnist_examples/models/cnn.py:31-120``).

conv5x5(1->32, same) -> ReLU -> maxpool2 -> conv5x5(32->64, same) -> ReLU ->
maxpool2 -> FC 3136->2048 -> ReLU -> FC 2048->10; cross-entropy on logits;
Adam(lr=1e-3).  6,497,162 parameters, same names as the reference
(``conv1``, ``conv2``, ``l1``, ``l2``).

This module is the eager/torch definition.  On MI355X the
:class:`~p2pfl_amd.learning.fused_cnn.FusedCNNLearner` runs the same
parameters through hand-written HIP kernels (see ``csrc/cnn_*.hip``).
"""

from __future__ import annotations

from typing import Optional

import torch
from torch import nn

from p2pfl_amd.models.base import FLModule, seed_everything

IMAGE_SIZE = 28


class CNN(FLModule):
    def __init__(
        self, in_channels: int = 1, out_channels: int = 10, lr_rate: float = 0.001, seed: Optional[int] = None
    ) -> None:
        seed_everything(seed)
        super().__init__()
        self.lr_rate = lr_rate
        self.conv1 = nn.Conv2d(in_channels, 32, kernel_size=(5, 5), padding="same")
        self.relu = nn.ReLU()
        self.pool1 = nn.MaxPool2d(kernel_size=(2, 2), stride=2)
        self.conv2 = nn.Conv2d(32, 64, kernel_size=(5, 5), padding="same")
        self.pool2 = nn.MaxPool2d(kernel_size=(2, 2), stride=2)
        self.l1 = nn.Linear(7 * 7 * 64, 2048)
        self.l2 = nn.Linear(2048, out_channels)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = x.reshape(-1, 1, IMAGE_SIZE, IMAGE_SIZE)
        x = self.pool1(self.relu(self.conv1(x)))
        x = self.pool2(self.relu(self.conv2(x)))
        x = x.reshape(-1, 7 * 7 * 64)
        x = self.relu(self.l1(x))
        return self.l2(x)
