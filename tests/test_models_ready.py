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
    cmd.execute("mem://b", 4)  # ahead of us: ignored
    cmd.execute("mem://c", 0)  # two or more rounds late: ignored (reference window r-1, r)
    assert "mem://b" not in state.nei_status and "mem://c" not in state.nei_status
    monkeypatch.setattr(Settings, "ASYNC_DIFFUSION", True)
    cmd.execute("mem://c", 0)  # background diffusion keeps any older round
    assert state.nei_status["mem://c"] == 0


def test_not_running_is_ignored():
    s = NodeState("mem://me")
    s.round = None
    ModelsReadyCommand(s).execute("mem://a", 1)
    assert s.nei_status == {}
