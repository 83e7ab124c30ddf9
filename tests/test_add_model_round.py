"""The models_aggregated report of an add_model carries the round of the models it lists.

Race found with 8 virtual peers (bench_node.py): the add that completes a node's
aggregation lets its learning thread advance the round before the command handler
broadcasts the report; stamped with the new round, the report was ignored by every peer
still in the old round, which kept offering models until their gossip loop's
equal-rounds exit (9 s stalls).  Reference behaviour being fixed:
/root/reference/p2pfl/commands/add_model_command.py:88-100.
"""

from __future__ import annotations

from types import SimpleNamespace

from p2pfl_amd.commands.add_model_command import AddModelCommand
from p2pfl_amd.commands.models_agregated_command import ModelsAggregatedCommand


class _Changed:
    def bump(self) -> None:
        pass


def test_report_keeps_the_round_of_the_added_models():
    sent = []
    state = SimpleNamespace(round=8, train_set=["a", "b"], learner=None, changed=_Changed(), addr="a")

    class Agg:
        def would_accept(self, contributors):
            return True

        def add_model(self, params, contributors, weight):
            state.round = 9  # the learning thread finished the round meanwhile
            return ["a", "b"]

    class Learner:
        def decode_parameters(self, w):
            return w

    class Proto:
        def build_msg(self, cmd, args=None, round=None):
            return (cmd, list(args or []), round)

        def broadcast(self, msg, node_list=None):
            sent.append(msg)

    state.learner = Learner()
    cmd = AddModelCommand(state, stop=lambda: None, aggregator=Agg(), comm_proto=Proto())
    cmd.execute("b", 8, weights={"w": 1}, contributors=["b"], weight=1)
    assert sent == [(ModelsAggregatedCommand.get_name(), ["a", "b"], 8)]


def test_stale_report_does_not_shrink_a_newer_one():
    """Reports of one round arrive out of order (two adds broadcast from concurrent
    handler threads): the 7-model report landing after the 8-model one must not make
    this node believe the peer lacks a model (it pushed until its equal-rounds exit)."""
    state = SimpleNamespace(round=1, models_aggregated={}, changed=_Changed(), addr="x")
    cmd = ModelsAggregatedCommand(state)
    full = [f"n{i}" for i in range(8)]
    cmd.execute("n0", 1, *full)
    cmd.execute("n0", 1, *full[:7])
    assert sorted(state.models_aggregated["n0"]) == sorted(full)
    cmd.execute("n0", 0, "late")  # another round's report is still ignored
    assert "late" not in state.models_aggregated["n0"]
