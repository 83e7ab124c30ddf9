"""Repro helper: tests/test_gpu_node.py::test_virtual_peers_on_gpu (3 virtual CNN peers on one
GPU, in-memory transport), repeated, with DEBUG logging so a learner error prints its traceback.

    python scripts/repro_virtual_peers.py [--reps 3] [--model cnn|mlp]
"""

from __future__ import annotations

import argparse
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--model", default="cnn")
    args = ap.parse_args()
    from p2pfl_amd import ops
    from p2pfl_amd.communication.memory import InMemoryCommunicationProtocol
    from p2pfl_amd.data import MnistFederatedDM
    from p2pfl_amd.models import CNN, MLP
    from p2pfl_amd.node import Node
    from p2pfl_amd.settings import Settings
    from p2pfl_amd.utils import check_equal_models, wait_4_results, wait_convergence

    Settings.LOG_LEVEL = "DEBUG"
    ops.ext()
    model = CNN if args.model == "cnn" else MLP
    for rep in range(args.reps):
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
            print(f"[repro] rep {rep}: OK ({type(nodes[0].state.learner).__name__})", flush=True)
        except Exception:
            traceback.print_exc()
            print(f"[repro] rep {rep}: FAILED", flush=True)
            sys.exit(1)
        finally:
            for nd in nodes:
                nd.stop()


if __name__ == "__main__":
    main()
