"""End-to-end node tests (reference ``test/node_test.py``) on both transports."""

from __future__ import annotations

import time

import pytest

from p2pfl_amd.data import MnistFederatedDM
from p2pfl_amd.exceptions import LearnerNotSetException, NodeRunningException, ZeroRoundsException
from p2pfl_amd.models import CNN, MLP
from p2pfl_amd.node import Node
from p2pfl_amd.utils import check_equal_models, wait_4_results, wait_convergence


def _chain(protocol, n, model=MLP, epochs_data=40):
    nodes = []
    for i in range(n):
        nd = Node(model(seed=i), MnistFederatedDM(sub_id=i % epochs_data, number_sub=epochs_data), protocol=protocol)
        nd.start()
        nodes.append(nd)
    for i in range(n - 1):
        nodes[i + 1].connect(nodes[i].addr)
    wait_convergence(nodes, n - 1, only_direct=False, wait=10)
    return nodes


@pytest.mark.parametrize("n,r", [(2, 1), (2, 2), (4, 2)])
def test_convergence(protocol, n, r):
    nodes = _chain(protocol, n)
    try:
        nodes[0].set_start_learning(rounds=r, epochs=0)
        wait_4_results(nodes, timeout=90)
        check_equal_models(nodes)
    finally:
        for nd in nodes:
            nd.stop()


def test_convergence_with_training_learns(protocol):
    """Real local SGD: federated model improves and all peers agree."""
    from p2pfl_amd.management.logger import logger

    nodes = _chain(protocol, 3)
    try:
        nodes[0].set_start_learning(rounds=2, epochs=1)
        wait_4_results(nodes, timeout=120)
        check_equal_models(nodes, atol=1e-5)
        logs = logger.get_global_logs()["experiment"]
        for nd in nodes:
            acc = dict(logs[nd.addr]["test_metric"])
            assert acc[2] > acc[0] + 0.2
    finally:
        for nd in nodes:
            nd.stop()


def test_train_set_smaller_than_network(protocol):
    """TRAIN_SET_SIZE < peers: non-members only receive the diffused aggregate."""
    from p2pfl_amd.settings import Settings

    old = Settings.TRAIN_SET_SIZE
    Settings.TRAIN_SET_SIZE = 2
    nodes = _chain(protocol, 4)
    try:
        nodes[0].set_start_learning(rounds=2, epochs=0)
        wait_4_results(nodes, timeout=90)
        check_equal_models(nodes)
    finally:
        Settings.TRAIN_SET_SIZE = old
        for nd in nodes:
            nd.stop()


def test_interrupt_train(protocol):
    """``set_stop_learning`` mid-experiment stops every node (reference test never ran its body: Q16)."""
    nodes = _chain(protocol, 2)
    try:
        nodes[0].set_start_learning(rounds=100, epochs=100)
        time.sleep(1.0)
        assert any(nd.state.round is not None for nd in nodes)
        nodes[0].set_stop_learning()
        wait_4_results(nodes, timeout=30)
    finally:
        for nd in nodes:
            nd.stop()


@pytest.mark.parametrize("n", [2, 4])
def test_node_down_on_learning(protocol, n):
    nodes = _chain(protocol, n)
    try:
        nodes[0].set_start_learning(rounds=2, epochs=0)
        time.sleep(0.3)
        nodes[-1].stop()
        wait_4_results(nodes, timeout=90)
    finally:
        for nd in nodes:
            nd.stop()


def test_wrong_model(protocol):
    n1 = Node(MLP(), MnistFederatedDM(number_sub=40), protocol=protocol)
    n2 = Node(CNN(), MnistFederatedDM(number_sub=40), protocol=protocol)
    n1.start()
    n2.start()
    try:
        n1.connect(n2.addr)
        wait_convergence([n1, n2], 1, only_direct=True)
        n1.set_start_learning(rounds=2, epochs=0)
        wait_4_results([n1, n2], timeout=90)
        # the CNN node refused the MLP weights and stopped itself
        with pytest.raises(NodeRunningException):
            n2.assert_running(True)
    finally:
        n1.stop()
        n2.stop()


def test_node_api_guards(protocol):
    n = Node(MLP(), MnistFederatedDM(number_sub=40), protocol=protocol)
    with pytest.raises(NodeRunningException):
        n.connect("127.0.0.1:1")
    n.start()
    with pytest.raises(NodeRunningException):
        n.start()
    with pytest.raises(ZeroRoundsException):
        n.set_start_learning(rounds=0)
    n.set_model(MLP())
    n.state.learner = object()
    with pytest.raises(LearnerNotSetException):
        n.set_data(None)
    n.state.learner = None
    n.stop()


def test_non_iid_and_dirichlet_partitions():
    from p2pfl_amd.data import FederatedDataModule

    ls = MnistFederatedDM(sub_id=0, number_sub=5, iid=False)
    labels = ls.train_dataloader().y.unique().tolist()
    assert len(labels) <= 3
    d0 = FederatedDataModule.from_dataset("mnist", 0, 4, partitioner="dirichlet", alpha=0.1, seed=3)
    d1 = FederatedDataModule.from_dataset("mnist", 1, 4, partitioner="dirichlet", alpha=0.1, seed=3)
    h0 = d0.train_dataloader().y.bincount(minlength=10).float()
    h1 = d1.train_dataloader().y.bincount(minlength=10).float()
    assert (h0 / h0.sum() - h1 / h1.sum()).abs().sum() > 0.5  # strongly skewed


def test_partial_neighbourhood_gossip_with_peer_dropped_mid_round(protocol):
    """BASELINE config 5 on the CPU: ring topology (each node sees 2 direct
    neighbours), train set of 4 out of 6, a train-set member stops while the
    round is training; the survivors finish all rounds with one model."""
    from p2pfl_amd.settings import Settings

    old = (Settings.TRAIN_SET_SIZE, Settings.GOSSIP_MODELS_PER_ROUND)
    Settings.TRAIN_SET_SIZE, Settings.GOSSIP_MODELS_PER_ROUND = 4, 2
    n = 6
    nodes = []
    try:
        for i in range(n):
            nd = Node(MLP(seed=i), MnistFederatedDM(sub_id=i, number_sub=n * 4), protocol=protocol)
            nd.start()
            nodes.append(nd)
        for i in range(n):  # ring
            nodes[i].connect(nodes[(i + 1) % n].addr)
        wait_convergence(nodes, n - 1, only_direct=False, wait=20)
        assert all(len(nd.get_neighbors(only_direct=True)) == 2 for nd in nodes)
        nodes[0].set_start_learning(rounds=3, epochs=1)
        t0 = time.time()
        while not nodes[0].state.train_set:
            assert time.time() - t0 < 60, "vote never finished"
            time.sleep(0.01)
        victim = next(nd for nd in nodes[1:] if nd.addr in nodes[0].state.train_set)
        time.sleep(0.05)
        victim.stop()
        survivors = [nd for nd in nodes if nd is not victim]
        wait_4_results(survivors, timeout=180)
        check_equal_models(survivors)
        acc = survivors[0].state.learner.evaluate()["test_metric"]
        assert acc > 0.6, acc
    finally:
        Settings.TRAIN_SET_SIZE, Settings.GOSSIP_MODELS_PER_ROUND = old
        for nd in nodes:
            nd.stop()
