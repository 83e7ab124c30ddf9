"""Model zoo: reference MNIST models plus the BASELINE target architectures."""

from p2pfl_amd.models.base import FLModule, seed_everything
from p2pfl_amd.models.cnn import CNN
from p2pfl_amd.models.mlp import MLP

__all__ = ["FLModule", "seed_everything", "CNN", "MLP"]
