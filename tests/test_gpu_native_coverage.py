"""Whole training rounds of the BASELINE configs on the hand-written kernels only.

Every convolution and Linear product of a ResNet-18 / ResNet-50 / ViT fit() -- eager
first steps, captured step graphs, the ragged last batch of the epoch and the
evaluation passes -- must run on csrc/ kernels: with ``P2PFL_STRICT_NATIVE`` on, a
shape the native kernels refuse raises instead of falling back to MIOpen / hipBLASLt,
and the fallback counters stay at zero.  (Reference models being replaced:
/root/reference/p2pfl/learning/pytorch/mnist_examples/models/cnn.py:55-71.)
"""

from __future__ import annotations

import importlib

import pytest
import torch

from p2pfl_amd import ops

pytestmark = pytest.mark.gpu

conv_mod = importlib.import_module("p2pfl_amd.ops.conv")
gemm_mod = importlib.import_module("p2pfl_amd.ops.gemm")


@pytest.fixture(autouse=True)
def _strict(monkeypatch):
    ops.ext()
    monkeypatch.setattr(gemm_mod, "STRICT", True)
    for k in conv_mod.STATS:
        conv_mod.STATS[k] = 0
    for k in gemm_mod.STATS:
        gemm_mod.STATS[k] = 0


@pytest.mark.parametrize("arch", ["resnet18", "resnet50"])
def test_resnet_fit_runs_native_only(arch):
    from p2pfl_amd.data import Cifar10FederatedDM
    from p2pfl_amd.learning.torch_learner import TorchLearner
    from p2pfl_amd.models.resnet import ResNet18, ResNet50

    torch.manual_seed(0)
    make = ResNet18 if arch == "resnet18" else ResNet50
    data = Cifar10FederatedDM(sub_id=3, number_sub=150, batch_size=32)
    n = len(data.train_dataloader().dataset)
    assert n % 32, "the shard must end in a ragged batch"
    ln = TorchLearner(make(num_classes=10, seed=0), data, f"cov-{arch}", 1, device=torch.device("cuda"))
    for _ in range(2):  # the second fit replays the captured step graphs
        ln.fit()
        res = ln.evaluate()
    assert res and all(torch.isfinite(torch.tensor(v)) for v in res.values())
    assert conv_mod.STATS["torch_fwd"] == 0, conv_mod.STATS
    assert gemm_mod.STATS["torch"] == 0, gemm_mod.STATS
    assert conv_mod.STATS["native_fwd"] + conv_mod.STATS["gemm_1x1_fwd"] > 0


def test_vit_fit_runs_native_only():
    from p2pfl_amd.data import Cifar10FederatedDM
    from p2pfl_amd.learning.torch_learner import TorchLearner
    from p2pfl_amd.models.vit import ViT_Tiny

    torch.manual_seed(0)
    data = Cifar10FederatedDM(sub_id=0, number_sub=150, batch_size=32)
    # 16 classes: every Linear output a multiple of 8 (the CIFAR labels use 10 of them)
    ln = TorchLearner(ViT_Tiny(num_classes=16, seed=0), data, "cov-vit", 1, device=torch.device("cuda"))
    for _ in range(2):
        ln.fit()
        res = ln.evaluate()
    assert res and all(torch.isfinite(torch.tensor(v)) for v in res.values())
    assert gemm_mod.STATS["torch"] == 0, gemm_mod.STATS
