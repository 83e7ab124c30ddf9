"""BASELINE target architectures (ResNet-18/50, ViT) on the CPU plumbing path."""

from __future__ import annotations

import torch

from p2pfl_amd.learning.arena import ModuleArena
from p2pfl_amd.learning.optim import ArenaAdam, ArenaSGD
from p2pfl_amd.models.resnet import ResNet18, ResNet50
from p2pfl_amd.models.vit import ViT_B16, ViT_Tiny


def test_param_counts():
    assert sum(p.numel() for p in ResNet18(seed=0).parameters()) == 11_173_962
    assert sum(p.numel() for p in ViT_B16(seed=0).parameters()) == 86_567_656


def test_forward_shapes():
    x = torch.randint(0, 255, (2, 3, 32, 32), dtype=torch.uint8)
    assert ResNet18(seed=0)(x).shape == (2, 10)
    assert ResNet50(seed=0)(x).shape == (2, 10)
    assert ViT_Tiny(seed=0)(x).shape == (2, 10)
    assert ResNet18(num_classes=100, stem="imagenet", seed=0)(torch.randint(0, 255, (1, 3, 64, 64), dtype=torch.uint8)).shape == (1, 100)


def test_arena_optimizers_leave_batchnorm_buffers_alone():
    """Weight decay must not shrink BatchNorm running statistics that share the arena."""
    for make in (lambda a: ArenaSGD(a, lr=0.1, momentum=0.9, weight_decay=0.1), lambda a: ArenaAdam(a, lr=0.1, weight_decay=0.1, decoupled=True)):
        m = ResNet18(seed=0)
        m.train()
        m(torch.randint(0, 255, (4, 3, 32, 32), dtype=torch.uint8))  # populate running stats
        arena = ModuleArena(m, grads=True)
        bufs = {k: v.clone() for k, v in m.state_dict().items() if "running" in k or "num_batches" in k}
        w0 = m.conv1.weight.clone() if hasattr(m, "conv1") else m.stem[0].weight.clone()
        opt = make(arena)
        arena.grads.fill_(0.01)
        opt.step()
        for k, v in m.state_dict().items():
            if k in bufs:
                assert torch.equal(v, bufs[k]), k
        assert not torch.equal(m.stem[0].weight, w0)


def test_resnet_learner_round_cpu():
    from p2pfl_amd.data import Cifar10FederatedDM
    from p2pfl_amd.learning.torch_learner import TorchLearner

    dm = Cifar10FederatedDM(sub_id=0, number_sub=100, batch_size=16)
    ln = TorchLearner(ResNet18(seed=0), dm, "r18", 1, device=torch.device("cpu"))
    before = ln.get_parameters().flat.clone()
    ln.fit()
    after = ln.get_parameters().flat
    assert not torch.equal(before, after)
    assert torch.isfinite(after).all()
    assert set(ln.evaluate()) == {"test_loss", "test_metric"}
