"""Full-stack round benchmark: K federated Nodes on one GPU, reference control plane.

Where ``bench.py`` times the data path of a FedAvg round (train + evaluate +
aggregate), this runs the whole p2pfl protocol end to end -- Node.start,
connect, set_start_learning, initial-model gossip, train-set vote, training,
partial-aggregate gossip, models_ready/diffusion, round bookkeeping -- with
the reference's DEFAULT ``Settings`` (gossip periods, heartbeats, timeouts).
The reference sleeps >= 2 s per round in its gossip loops
(``gossiper.py:242-243``, ``settings.py:76,104``); this build's control
plane is event-driven, so the periods are only upper bounds.

K virtual peers share one MI355X through the in-memory transport with
device-resident payloads (models never leave HBM); each peer trains the
reference CNN with the fused HIP engine on its own MNIST-shaped shard.

    python bench_node.py --peers 4 --rounds 5
Prints one JSON line: per-round wall clock (steady state = rounds 2..R),
time to first round, samples/s per peer, final test accuracy.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--peers", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--epochs", type=int, default=1)
    ap.add_argument("--number-sub", type=int, default=20)
    ap.add_argument("--learner", choices=["fused", "torch"], default="fused")
    ap.add_argument("--watchdog", type=float, default=600)
    ap.add_argument("--log-level", default="WARNING", help="node log level (INFO shows every stage / gossip step)")
    args = ap.parse_args()
    import faulthandler

    faulthandler.dump_traceback_later(args.watchdog, exit=True)

    from p2pfl_amd.communication.memory import InMemoryCommunicationProtocol
    from p2pfl_amd.data import MnistFederatedDM
    from p2pfl_amd.management.logger import logger
    from p2pfl_amd.models import CNN
    from p2pfl_amd.node import Node
    from p2pfl_amd.settings import Settings
    from p2pfl_amd.utils import wait_4_results, wait_convergence

    Settings.LOG_LEVEL = args.log_level
    Settings.TRAIN_SET_SIZE = max(Settings.TRAIN_SET_SIZE, args.peers)
    if args.learner == "fused":
        from p2pfl_amd.learning.fused_cnn import FusedCNNLearner as L
    else:
        from p2pfl_amd.learning.torch_learner import TorchLearner as L
    dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    nodes = []
    for i in range(args.peers):
        data = MnistFederatedDM(sub_id=i % args.number_sub, number_sub=args.number_sub)
        n = Node(CNN(seed=i), data, learner=L, protocol=InMemoryCommunicationProtocol, device=dev)
        n.start()
        nodes.append(n)
    try:
        for i in range(1, args.peers):
            nodes[i].connect(nodes[0].addr)
        wait_convergence(nodes, args.peers - 1, only_direct=False, wait=60)
        t0 = time.perf_counter()  # the tracer's clock
        nodes[0].set_start_learning(rounds=args.rounds, epochs=args.epochs)
        wait_4_results(nodes, timeout=args.watchdog)
        total = time.perf_counter() - t0
        ends = sorted(s.start + s.duration for s in logger.tracer.spans(nodes[0].addr, "stage:RoundFinishedStage"))
        per_round = [b - a for a, b in zip(ends, ends[1:])]
        steady = sum(per_round) / len(per_round) if per_round else total / args.rounds
        median = sorted(per_round)[len(per_round) // 2] if per_round else steady
        first = (ends[0] - t0) if ends else total
        n_train = len(nodes[0].data.train_dataloader().dataset)
        acc = nodes[0].state.learner.evaluate()["test_metric"] if nodes[0].state.learner else None
    finally:
        for n in nodes:
            n.stop()
    print(
        json.dumps(
            {
                "metric": "full-stack wall-clock per FedAvg round (steady state), reference default Settings",
                "value": round(steady * 1e3, 2),
                "unit": "ms/round",
                "higher_is_better": False,
                "peers": args.peers,
                "rounds": args.rounds,
                "median_round_ms": round(median * 1e3, 2),
                "rounds_ms": [round(x * 1e3, 2) for x in per_round],
                "first_round_ms": round(first * 1e3, 2),
                "total_s": round(total, 3),
                "samples_per_sec_per_peer": round(n_train * args.epochs / steady, 1),
                "final_test_accuracy": acc,
                "learner": args.learner,
                "device": str(dev),
                "config": "MNIST-CNN, batch 32, Adam 1e-3, 2700-sample shards, in-memory transport (device payloads), 1 GPU",
            }
        ),
        flush=True,
    )


if __name__ == "__main__":
    main()
