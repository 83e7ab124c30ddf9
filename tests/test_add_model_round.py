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
