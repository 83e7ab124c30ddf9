"""Partial-neighbourhood gossip with a peer dropped mid-round (BASELINE config 5).

K virtual peers on a ring (each sees 2 direct neighbours), a train set of
K/2 voted per experiment, ResNet on CIFAR-10-shaped Dirichlet shards (or the
MLP on MNIST for a quick CPU run); one train-set member is stopped while the
first round trains.  The survivors must finish every round with one shared
model; per-round wall-clock is printed.  The reference would wait
AGGREGATION_TIMEOUT (300 s) in every round for the dead member; here the
aggregators mark it lost as soon as the heartbeats drop it.
"""

from __future__ import annotations

import argparse
import json
import time

import torch


def main(argv=None) -> None:
    p = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    p.add_argument("--peers", type=int, default=8)
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--model", choices=["resnet50", "resnet18", "mlp"], default="resnet50")
    p.add_argument("--number-sub", type=int, default=64, help="dataset shards (per-peer data = 1/number-sub)")
    p.add_argument("--fast", action="store_true", help="test settings (short heartbeats)")
    p.add_argument("--lr", type=float, default=None, help="override the ResNet SGD learning rate (default 0.05)")
    p.add_argument("--no-step-graphs", action="store_true", help="eager training steps (no HIP-graph replay)")
    p.add_argument("--overlap", choices=["on", "off", "async", "streams"], default="on",
                   help="on: background diffusion (Settings.ASYNC_DIFFUSION) + per-node HIP streams; "
                        "off: the reference's blocking diffusion, all peers on the default stream; "
                        "async / streams: only one of the two")
    args = p.parse_args(argv)
    if args.no_step_graphs:
        import os

        os.environ["P2PFL_STEP_GRAPHS"] = "0"

    from p2pfl_amd.communication.memory import InMemoryCommunicationProtocol
    from p2pfl_amd.management.logger import logger
    from p2pfl_amd.node import Node
    from p2pfl_amd.settings import Settings
    from p2pfl_amd.utils import check_equal_models, set_test_settings, wait_4_results, wait_convergence

    if args.fast:
        set_test_settings()
    Settings.LOG_LEVEL = "WARNING"
    Settings.ASYNC_DIFFUSION = args.overlap in ("on", "async")
    Settings.NODE_STREAMS = args.overlap in ("on", "streams")
    Settings.TRAIN_SET_SIZE = max(2, args.peers // 2)
    Settings.GOSSIP_MODELS_PER_ROUND = 2
    dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    if args.model == "mlp":
        from p2pfl_amd.data import MnistFederatedDM
        from p2pfl_amd.models import MLP

        make = lambda i: (MLP(seed=i), MnistFederatedDM(sub_id=i, number_sub=args.number_sub))  # noqa: E731
    else:
        from p2pfl_amd.data import Cifar10FederatedDM
        from p2pfl_amd.models.resnet import ResNet18, ResNet50

        net = ResNet50 if args.model == "resnet50" else ResNet18
        kw = {} if args.lr is None else {"lr_rate": args.lr}
        make = lambda i: (  # noqa: E731
            net(seed=1234, **kw),
            Cifar10FederatedDM(sub_id=i, number_sub=args.number_sub, partitioner="dirichlet", alpha=0.5),
        )
    nodes = []
    for i in range(args.peers):
        model, data = make(i)
        n = Node(model, data, protocol=InMemoryCommunicationProtocol, device=dev)
        n.start()
        nodes.append(n)
    victim = None
    try:
        for i in range(args.peers):
            nodes[i].connect(nodes[(i + 1) % args.peers].addr)
        wait_convergence(nodes, args.peers - 1, only_direct=False, wait=60)
        t0 = time.perf_counter()
        nodes[0].set_start_learning(rounds=args.rounds, epochs=1)
        while not nodes[0].state.train_set:
            time.sleep(0.01)
        victim = next(n for n in nodes[1:] if n.addr in nodes[0].state.train_set)
        time.sleep(0.2)
        victim.stop()
        survivors = [n for n in nodes if n is not victim]
        from p2pfl_amd.utils import finite

        t_wait, t_print = time.monotonic(), 0.0
        while any(n.state.round is not None for n in survivors):
            if finite.FIRST_FAILURE:  # P2PFL_CHECK_FINITE=1: stop at the first non-finite tensor
                node, msg = finite.FIRST_FAILURE[0]
                print(json.dumps({"non_finite": True, "node": node, "error": msg}), flush=True)
                import os

                os._exit(3)
            if time.monotonic() - t_print > 10:  # progress (also keeps watchdogs fed)
                t_print = time.monotonic()
                print(f"[fault_tolerance] {time.monotonic() - t_wait:.0f}s: rounds "
                      f"{[n.state.round for n in survivors]}", flush=True)
            if time.monotonic() - t_wait > 1800:
                raise TimeoutError("survivors did not finish")
            time.sleep(0.05)
        wait_4_results(survivors, timeout=60)
        total = time.perf_counter() - t0
        try:
            check_equal_models(survivors)
        except AssertionError as e:
            torch.cuda.synchronize()  # every learner's stream (diagnostics only)
            ref = survivors[0].state.learner.get_parameters().flat
            for s_ in survivors:
                d = float((s_.state.learner.get_parameters().flat - ref).abs().max())
                rounds_done = len(logger.tracer.spans(s_.addr, "stage:RoundFinishedStage"))
                print(f"  {s_.addr}: max|diff| vs {survivors[0].addr} = {d:.3g}, rounds finished {rounds_done}, "
                      f"train_set member: {s_.addr in survivors[0].state.train_set}", flush=True)
            raise e
        ends = sorted(s.start + s.duration for s in logger.tracer.spans(survivors[0].addr, "stage:RoundFinishedStage"))
        rounds = [round((b - a) * 1e3, 1) for a, b in zip([t0] + ends, ends)]
        acc = survivors[0].state.learner.evaluate()["test_metric"]
    finally:
        for n in nodes:
            n.stop()
    print(json.dumps({
        "scenario": "ring topology, train set K/2, 1 train-set peer dropped mid-round",
        "peers": args.peers, "model": args.model, "device": str(dev), "dropped": victim.addr if victim else None,
        "overlap": args.overlap,
        "round_ms": rounds, "total_s": round(total, 2), "survivors_equal_models": True, "test_accuracy": acc,
    }), flush=True)


if __name__ == "__main__":
    main()
