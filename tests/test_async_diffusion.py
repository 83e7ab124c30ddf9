"""Background diffusion of a round's aggregate (Settings.ASYNC_DIFFUSION): the
next round trains while lagging neighbours still receive the previous
aggregate.  Same end states as the blocking (reference) diffusion."""

from __future__ import annotations

import time

import pytest

from p2pfl_amd.data import MnistFederatedDM
from p2pfl_amd.models import MLP
from p2pfl_amd.node import Node
from p2pfl_amd.settings import Settings
from p2pfl_amd.utils import check_equal_models, wait_4_results, wait_convergence


@pytest.fixture
def async_settings():
    old = (Settings.ASYNC_DIFFUSION, Settings.TRAIN_SET_SIZE, Settings.GOSSIP_MODELS_PER_ROUND)
    Settings.ASYNC_DIFFUSION = True
    yield
    Settings.ASYNC_DIFFUSION, Settings.TRAIN_SET_SIZE, Settings.GOSSIP_MODELS_PER_ROUND = old


def _start(n, protocol, subs):
    nodes = []
    for i in range(n):
        nd = Node(MLP(seed=i), MnistFederatedDM(sub_id=i, number_sub=subs), protocol=protocol)
        nd.start()
        nodes.append(nd)
    return nodes


def test_async_diffusion_chain_non_trainers(protocol, async_settings):
    """Train set of 2 on a 4-chain: the non-trainers only get the diffused
    aggregate, which now travels while the trainers start the next round."""
    Settings.TRAIN_SET_SIZE = 2
    nodes = _start(4, protocol, 40)
    try:
        for i in range(3):
            nodes[i + 1].connect(nodes[i].addr)
        wait_convergence(nodes, 3, only_direct=False, wait=10)
        nodes[0].set_start_learning(rounds=3, epochs=1)
        wait_4_results(nodes, timeout=120)
        check_equal_models(nodes, atol=1e-5)
        # every background diffusion has ended with the experiment
        for nd in nodes:
            assert all(not d.thread.is_alive() for d in getattr(nd.state, "diffusions", []))
    finally:
        for nd in nodes:
            nd.stop()


def test_async_diffusion_ring_with_peer_dropped(protocol, async_settings):
    """BASELINE config 5 with overlapped diffusion: ring of 6, train set 4,
    a train-set member stops mid-round; the survivors agree."""
    Settings.TRAIN_SET_SIZE, Settings.GOSSIP_MODELS_PER_ROUND = 4, 2
    n = 6
    nodes = _start(n, protocol, n * 4)
    try:
        for i in range(n):
            nodes[i].connect(nodes[(i + 1) % n].addr)
        wait_convergence(nodes, n - 1, only_direct=False, wait=20)
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
    finally:
        for nd in nodes:
            nd.stop()


def test_diffusion_payload_is_a_snapshot(async_settings):
    """The background diffusion pushes the aggregate captured when it started,
    even though the next round keeps training the live arena."""
    import torch

    from p2pfl_amd.stages.base_node.gossip_model_stage import Diffusion

    class _State:
        addr = "n0"
        round = 1
        nei_status = {"x": 0}  # one neighbour behind round 1

        class changed:  # noqa: N801
            version = 0

    class _Learner:
        def __init__(self):
            self.w = torch.zeros(4)

        def snapshot_parameters(self, params=None):
            return self.w.clone()

        def encode_parameters(self, params=None):
            return self.w.clone()

    class _Proto:
        supports_device_payloads = True
        sent = []

        def build_weights(self, cmd, rnd, payload, contributors, weight):
            return (rnd, payload, tuple(contributors))

        def get_neighbors(self, only_direct=False):
            return ["x"]

        def gossip_weights(self, stop, cands, status, model_fn, wakeup=None, peer_status_fn=None):
            self.sent.append(model_fn("x"))

    class _Agg:
        def get_aggregated_models(self):
            return ["n0", "n1"]

    st = _State()
    st.learner = _Learner()
    proto = _Proto()
    d = Diffusion.start(st, proto, _Agg(), 1)
    st.learner.w.add_(5.0)  # "next round" trains the live weights
    d.join(5)
    rnd, payload, contributors = proto.sent[0]
    assert rnd == 1 and contributors == ("n0", "n1")
    assert torch.equal(payload, torch.zeros(4))
