"""Start a gRPC node, connect it to node1's port and run 2 rounds of federated learning.

Reference: p2pfl/examples/node2.py.  ``python -m p2pfl_amd.examples.node2 6667 6666``
"""

from __future__ import annotations

import argparse

from p2pfl_amd.data import MnistFederatedDM
from p2pfl_amd.models import MLP
from p2pfl_amd.node import Node
from p2pfl_amd.utils import wait_convergence


def main(argv=None) -> None:
    p = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    p.add_argument("self_port", type=int, help="port to listen on")
    p.add_argument("port", type=int, help="node1's port")
    p.add_argument("--rounds", type=int, default=2)
    p.add_argument("--epochs", type=int, default=1)
    args = p.parse_args(argv)
    node = Node(MLP(), MnistFederatedDM(sub_id=1, number_sub=2), address=f"127.0.0.1:{args.self_port}")
    node.start()
    try:
        node.connect(f"127.0.0.1:{args.port}")
        wait_convergence([node], 1, only_direct=True)
        node.set_start_learning(rounds=args.rounds, epochs=args.epochs)
        node.wait_learning()
        learner = node.state.learner
        print(f"node2 finished: {learner.evaluate() if learner is not None else {}}", flush=True)
    finally:
        node.stop()


if __name__ == "__main__":
    main()
