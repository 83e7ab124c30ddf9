"""MNIST MLP 784-256-128-10 (reference ``mnist_examples/models/mlp.py:29-102``).

Same layer names (``l1``, ``l2``, ``l3``) so state-dict keys and the wire layout
match the reference.  ``forward`` returns log-probabilities and the loss is
cross-entropy on them (a double log-softmax, idempotent: quirk Q21 kept).
"""

from __future__ import annotations

from typing import Optional

import torch
from torch import nn

from p2pfl_amd.models.base import FLModule, seed_everything


class MLP(FLModule):
    def __init__(self, out_channels: int = 10, lr_rate: float = 0.001, seed: Optional[int] = None) -> None:
        seed_everything(seed)
        super().__init__()
        self.lr_rate = lr_rate
        self.l1 = nn.Linear(28 * 28, 256)
        self.l2 = nn.Linear(256, 128)
        self.l3 = nn.Linear(128, out_channels)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = x.reshape(x.shape[0], -1)
        if x.is_cuda:
            from p2pfl_amd import ops

            if ops.available():
                # 784->256 and 256->128 on the hand-written MFMA GEMM (bias in its epilogue)
                x = torch.relu(ops.linear(x, self.l1.weight, self.l1.bias))
                x = torch.relu(ops.linear(x, self.l2.weight, self.l2.bias))
                return torch.log_softmax(self.l3(x), dim=1)
        x = torch.relu(self.l1(x))
        x = torch.relu(self.l2(x))
        return torch.log_softmax(self.l3(x), dim=1)
