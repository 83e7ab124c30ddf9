"""On-disk checkpoints: flat arena + manifest (new; the reference has none -- SURVEY §5)."""

from __future__ import annotations

import os

import pytest
import torch

from p2pfl_amd.communication.memory import InMemoryCommunicationProtocol
from p2pfl_amd.data import MnistFederatedDM
from p2pfl_amd.learning.arena import flatten
from p2pfl_amd.learning.checkpoint import CheckpointError, load_checkpoint, save_checkpoint
from p2pfl_amd.models import CNN, MLP
from p2pfl_amd.node import Node
from p2pfl_amd.settings import Settings
from p2pfl_amd.utils import check_equal_models, wait_4_results, wait_convergence


def test_roundtrip_bitwise(tmp_path):
    m = MLP(seed=3)
    p = str(tmp_path / "a.safetensors")
    save_checkpoint(p, m.state_dict(), {"round": 4}, extra={"adam_m": torch.arange(5.0)})
    params, meta, extra = load_checkpoint(p)
    assert meta == {"round": 4}
    assert list(params) == list(m.state_dict())
    for a, b in zip(params.values(), m.state_dict().values()):
        assert torch.equal(a, b)
    assert torch.equal(extra["adam_m"], torch.arange(5.0))
    assert not [f for f in os.listdir(tmp_path) if f.endswith(".tmp")]


def test_shape_mismatch_and_garbage(tmp_path):
    p = str(tmp_path / "mlp.safetensors")
    save_checkpoint(p, MLP().state_dict())
    with pytest.raises(CheckpointError):
        load_checkpoint(p, expect=flatten(CNN().state_dict()).layout)
    bad = tmp_path / "bad.safetensors"
    bad.write_bytes(b"\x00" * 64)
    with pytest.raises(CheckpointError):
        load_checkpoint(str(bad))


def test_node_save_load_and_auto_checkpoint(tmp_path, monkeypatch):
    monkeypatch.setattr(Settings, "CHECKPOINT_DIR", str(tmp_path / "auto"))
    nodes = [Node(MLP(seed=i), MnistFederatedDM(sub_id=i, number_sub=4), protocol=InMemoryCommunicationProtocol) for i in range(2)]
    for n in nodes:
        n.start()
    try:
        nodes[1].connect(nodes[0].addr)
        wait_convergence(nodes, 1, only_direct=True)
        nodes[0].set_start_learning(rounds=2, epochs=1)
        wait_4_results(nodes, timeout=120)
        check_equal_models(nodes)
        ck = nodes[0].save_checkpoint(str(tmp_path / "final.safetensors"))
    finally:
        for n in nodes:
            n.stop()
    # one file per node and round
    for n in nodes:
        d = os.path.join(tmp_path, "auto", n.addr.replace("://", "_").replace("/", "_").replace(":", "_"))
        assert sorted(os.listdir(d)) == ["round_0.safetensors", "round_1.safetensors"], os.listdir(d)
    # resume: a fresh node loads the final model before learning
    fresh = Node(MLP(seed=99), MnistFederatedDM(sub_id=0, number_sub=4), protocol=InMemoryCommunicationProtocol)
    meta = fresh.load_checkpoint(ck)
    assert meta["addr"] == nodes[0].addr
    want = nodes[0].state.learner.get_parameters()
    for a, b in zip(fresh.model.state_dict().values(), want.values()):
        assert torch.allclose(a, b.cpu())
