"""``models_ready`` bookkeeping (commands/models_ready_command.py).

The reference records the receiver's own round for the sender (quirk Q12); a
neighbour one round behind then looks up to date and the aggregate's diffusion
skips it.  This build records the round the neighbour reported."""

from __future__ import annotations

import pytest

from p2pfl_amd.commands.models_ready_command import ModelsReadyCommand
from p2pfl_amd.node_state import NodeState
from p2pfl_amd.settings import Settings


@pytest.fixture
def state():
    s = NodeState("mem://me")
    s.round = 3
    return s


@pytest.mark.parametrize("async_diffusion", [False, True])
def test_previous_round_ready_is_recorded_as_reported(state, monkeypatch, async_diffusion):
    monkeypatch.setattr(Settings, "ASYNC_DIFFUSION", async_diffusion)
    cmd = ModelsReadyCommand(state)
    cmd.execute("mem://a", 2)  # a neighbour still finishing round 2
    assert state.nei_status["mem://a"] == 2  # still a diffusion candidate for round 3 (2 < 3)
    cmd.execute("mem://a", 3)
    assert state.nei_status["mem://a"] == 3
    cmd.execute("mem://a", 2)  # a late duplicate never moves the status back
    assert state.nei_status["mem://a"] == 3


def test_rounds_outside_the_window(state, monkeypatch):
    monkeypatch.setattr(Settings, "ASYNC_DIFFUSION", False)
    cmd = ModelsReadyCommand(state)
    cmd.execute("mem://b", 4)  # ahead of us: recorded (it needs nothing of round 3 any more)
    cmd.execute("mem://c", 0)  # two or more rounds late: ignored (reference window r-1, r)
    assert state.nei_status["mem://b"] == 4 and "mem://c" not in state.nei_status
    monkeypatch.setattr(Settings, "ASYNC_DIFFUSION", True)
    cmd.execute("mem://c", 0)  # background diffusion keeps any older round
    assert state.nei_status["mem://c"] == 0


def test_not_running_is_ignored():
    s = NodeState("mem://me")
    s.round = None
    ModelsReadyCommand(s).execute("mem://a", 1)
    assert s.nei_status == {}


def test_sync_diffusion_ends_by_stall_exit_when_a_neighbour_stays_behind(monkeypatch):
    """Blocking (reference) diffusion with the reported-round bookkeeping: a
    direct neighbour that keeps reporting round r - 1 stays a candidate, and the
    diffusion ends through the GOSSIP_EXIT_ON_X_EQUAL_ROUNDS stall exit after
    that many unchanged snapshots (one push per GOSSIP_MODELS_PERIOD meanwhile),
    not by hanging (ADVICE r4, Q12 parity break)."""
    import time

    from p2pfl_amd.communication.gossiper import Gossiper
    from p2pfl_amd.communication.messages import WeightsMessage
    from p2pfl_amd.stages.base_node.gossip_model_stage import GossipModelStage

    monkeypatch.setattr(Settings, "ASYNC_DIFFUSION", False)
    monkeypatch.setattr(Settings, "GOSSIP_EXIT_ON_X_EQUAL_ROUNDS", 3)
    monkeypatch.setattr(Settings, "GOSSIP_MODELS_PERIOD", 0.05)
    monkeypatch.setattr(Settings, "GOSSIP_MODELS_PER_ROUND", 2)
    st = NodeState("mem://me")
    st.round = 3
    st.train_set = ["mem://me", "mem://t"]
    ModelsReadyCommand(st).execute("mem://lag", 2)  # the lagging neighbour reports round 2, forever

    class _Learner:
        def snapshot_parameters(self, params=None):
            return b"w"

    st.learner = _Learner()
    sent = []

    class _Client:
        def send(self, nei, msg, create_connection=False):
            sent.append((nei, time.monotonic()))

    class _Proto:
        supports_device_payloads = True
        _gossiper = Gossiper("mem://me", _Client())

        def get_neighbors(self, only_direct=False):
            return ["mem://lag"]

        def build_weights(self, cmd, rnd, payload, contributors, weight):
            return WeightsMessage("mem://me", rnd, payload, list(contributors), weight, cmd)

        def gossip_weights(self, *a, **k):
            from p2pfl_amd.communication.protocol import BaseCommunicationProtocol

            return BaseCommunicationProtocol.gossip_weights(self, *a, **k)

    class _Agg:
        def get_aggregated_models(self):
            return ["mem://me", "mem://t"]

        def live_train_set(self):
            return ["mem://me", "mem://t"]

    t0 = time.monotonic()
    GossipModelStage._gossip_model_diffusion(st, _Proto(), _Agg())
    took = time.monotonic() - t0
    assert st.nei_status["mem://lag"] == 2
    assert 1 <= len(sent) <= 5 and all(n == "mem://lag" for n, _ in sent), sent
    assert took < 2.0, took  # 3 equal snapshots one period apart, then out


def test_partial_gossip_skips_a_peer_already_past_the_round():
    """TrainStage's partial-aggregate gossip: a peer whose models_ready says it has this
    round's aggregate is no candidate even if its last models_aggregated report of the
    round never arrived (it was sent while this node was still in the previous round).
    Before, the loop kept offering it models it declined until the equal-rounds exit
    (~9 s stalls with 8 virtual peers, bench_node.py)."""
    from p2pfl_amd.stages.base_node.train_stage import TrainStage

    st = NodeState("mem://me")
    st.round = 5
    st.train_set = ["mem://me", "mem://a", "mem://b"]
    st.models_aggregated = {"mem://a": ["mem://a"], "mem://b": ["mem://b"]}  # stale reports
    seen = {}

    class Agg:
        def get_aggregated_models(self):
            return ["mem://me", "mem://a", "mem://b"]

    class Proto:
        def get_neighbors(self, only_direct=False):
            return {"mem://a": None, "mem://b": None}

        def gossip_weights(self, stop, candidates, status, model_fn, **kw):
            seen["before"] = sorted(candidates())
            ModelsReadyCommand(st).execute("mem://a", 5)  # a finished round 5
            ModelsReadyCommand(st).execute("mem://b", 6)  # b is already past it
            seen["after"] = sorted(candidates())

    TrainStage._gossip_model_aggregation(st, Proto(), Agg())
    assert seen == {"before": ["mem://a", "mem://b"], "after": []}
