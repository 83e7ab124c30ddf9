"""Virtual peers sharing one MI355X: device payloads + HIP FedAvg/optimizer kernels end to end."""

from __future__ import annotations

import pytest
import torch

from p2pfl_amd import ops
from p2pfl_amd.communication.memory import InMemoryCommunicationProtocol
from p2pfl_amd.data import MnistFederatedDM
from p2pfl_amd.models import CNN, MLP
from p2pfl_amd.node import Node
from p2pfl_amd.utils import check_equal_models, wait_4_results, wait_convergence

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("model", [MLP, CNN])
def test_virtual_peers_on_gpu(model):
    ops.ext()
    nodes = []
    for i in range(3):
        nd = Node(model(seed=i), MnistFederatedDM(sub_id=i, number_sub=30), protocol=InMemoryCommunicationProtocol)
        nd.start()
        nodes.append(nd)
    try:
        for i in range(2):
            nodes[i + 1].connect(nodes[i].addr)
        wait_convergence(nodes, 2, only_direct=False)
        nodes[0].set_start_learning(rounds=2, epochs=1)
        wait_4_results(nodes, timeout=300)
        check_equal_models(nodes, atol=1e-6)
        for nd in nodes:
            params = nd.state.learner.get_parameters()
            assert params.flat.is_cuda
    finally:
        for nd in nodes:
            nd.stop()
