"""Model base class.

PyTorch Lightning is not part of this stack (and not installed); models are
plain ``nn.Module`` subclasses exposing the same hooks the reference's
LightningModules do (``training_step``, ``validation_step``, ``test_step``,
``configure_optimizers``, ``self.log``), so a reference model definition ports
by changing its base class.  The learner drives them.
"""

from __future__ import annotations

from typing import Any, Dict, Optional, Tuple

import torch
from torch import nn


class FLModule(nn.Module):
    """``nn.Module`` with Lightning-style step hooks and metric logging."""

    lr_rate: float = 1e-3

    def __init__(self) -> None:
        super().__init__()
        self._logged: Dict[str, Any] = {}

    # -- logging -----------------------------------------------------------
    def log(self, name: str, value: Any, prog_bar: bool = False, **kwargs) -> None:
        self._logged[name] = value.detach() if isinstance(value, torch.Tensor) else value

    def pop_logged(self) -> Dict[str, Any]:
        out, self._logged = self._logged, {}
        return out

    # -- hooks ---------------------------------------------------------------
    def loss_fn(self, out: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
        return nn.functional.cross_entropy(out, y)

    def configure_optimizers(self) -> torch.optim.Optimizer:
        return torch.optim.Adam(self.parameters(), lr=self.lr_rate)

    # True: forward() takes the raw uint8 batch and folds the /255 into its first
    # kernel (the learners then skip the float normalisation pass of the loader)
    takes_uint8 = False

    def training_step(self, batch: Tuple[torch.Tensor, torch.Tensor], batch_idx: int) -> torch.Tensor:
        x, y = batch
        loss = self.loss_fn(self(x), y)
        self.log("train_loss", loss, prog_bar=True)
        return loss

    def _eval_step(self, batch: Tuple[torch.Tensor, torch.Tensor], prefix: str) -> torch.Tensor:
        # The reference runs the forward twice per eval step (quirk Q21); once is enough.
        x, y = batch
        out = self(x)
        loss = self.loss_fn(out, y)
        acc = (out.argmax(dim=1) == y).float().mean()
        self.log(f"{prefix}_loss", loss, prog_bar=True)
        self.log(f"{prefix}_metric", acc, prog_bar=True)
        return loss

    def validation_step(self, batch: Tuple[torch.Tensor, torch.Tensor], batch_idx: int) -> torch.Tensor:
        return self._eval_step(batch, "val")

    def test_step(self, batch: Tuple[torch.Tensor, torch.Tensor], batch_idx: int) -> torch.Tensor:
        return self._eval_step(batch, "test")


def seed_everything(seed: Optional[int]) -> None:
    if seed is not None:
        torch.manual_seed(seed)
        if torch.cuda.is_available():
            torch.cuda.manual_seed_all(seed)
