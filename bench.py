"""Headline benchmark: MNIST-CNN FedAvg rounds, one federated peer (Node) per GPU.

Metric (BASELINE.json): wall-clock per round + samples/s per peer, MNIST-CNN
FedAvg at 1/2/4/8 peers.  ``value`` is the whole-job aggregate training
throughput (train samples/s summed over peers); ``ms_per_step`` is the
wall-clock of one federated round.

What runs: every rank is a full p2pfl
:class:`~p2pfl_amd.node.Node` driven through the reference's stage machine
(``Node.set_start_learning`` -> StartLearning -> VoteTrainSet -> Train ->
GossipModel -> RoundFinished, reference ``node.py:297-364``) on the xGMI
transport: control messages on the node-local bus, model pushes as RCCL
point-to-point transfers over xGMI (epoch-grouped, k-way link-parallel
fan-out), FedAvg of the received arenas by the hand-written HIP
``weighted_sum`` kernel.  Each round per peer (weak scaling, fixed per-peer
work): evaluate(test) -> fit(1 epoch + val) -> push partial aggregates to the
train set -> FedAvg -> models_ready / diffusion.  Full-mesh deployment
settings: train set = all peers, fan-out ``GOSSIP_MODELS_PER_ROUND = N-1``
(one push per xGMI link), ``TTL = 1`` (every peer is a direct neighbour, so
flooding adds no reachability); everything else is the reference default.

Timing: rounds run autonomously in each node's learning thread; a round hook
synchronises the GPU and takes a barrier across ranks after round W (start)
and after round W+K (end); the MAX over ranks of the bracketed time is
reported.

Per-peer round work matches the reference example shard
(``MnistFederatedDM(sub_id, number_sub=20)``): 2,700 train / 300 val / 500
test MNIST-shaped samples, batch 32, the reference CNN (6.5 M params), Adam
1e-3 re-created per round, 1 local epoch.

Other modes: ``--impl torch`` (the generic TorchLearner instead of the fused
CNN engine), ``--model resnet18|resnet50|vit_b16`` (BASELINE configs 3-5).  The
reference-equivalent baseline (fp32 eager, pickle, per-layer FedAvg) is measured
by ``scripts/reference_baseline.py``.

Launch: ``python bench.py --gpus N`` starts N worker processes itself (the
launcher never touches the GPU); under ``torchrun`` each process is one rank.
"""

from __future__ import annotations

import argparse
import json
import os
import signal
import socket
import subprocess
import sys
import time
import uuid

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

from p2pfl_amd.data import MnistFederatedDM  # noqa: E402
from p2pfl_amd.models import CNN  # noqa: E402

# Reference-equivalent baseline, measured (not published -- the reference
# publishes no timing): `python scripts/reference_baseline.py` (round 1:
# `bench.py --impl reference`) on one MI355X, 99.6 ms per round = 27,120.7 train samples/s per
# peer.  vs_baseline compares per-peer throughput with it; it is
# context, not a published comparison (the reference's own control plane
# sleeps >= 2 s per round on top of that work).
BASELINE_SAMPLES_PER_SEC_PER_PEER = 27120.7


# ----------------------------------------------------------------------------
# configs
# ----------------------------------------------------------------------------
def build_config(args, rank):
    """(model, data module, model description, data description) for ``--model``."""
    if args.model == "cnn":
        ns = args.number_sub or 20
        data = MnistFederatedDM(sub_id=rank % ns, number_sub=ns, batch_size=args.batch)
        return (
            CNN(seed=1234),
            data,
            "MNIST-CNN (p2pfl CNN: conv5x5 32/64 + FC 3136-2048-10, 6.5M params), Adam 1e-3",
            "synthetic MNIST-shaped (uint8 1x28x28, 10 classes), random-init weights",
        )
    if args.model in ("resnet18", "resnet50"):
        from p2pfl_amd.data import Cifar10FederatedDM
        from p2pfl_amd.models.resnet import ResNet18, ResNet50

        ns = args.number_sub or 40
        data = Cifar10FederatedDM(sub_id=rank % ns, number_sub=ns, batch_size=args.batch, partitioner="dirichlet", alpha=0.5)
        make = ResNet18 if args.model == "resnet18" else ResNet50
        n = "ResNet-18 (11.2M params)" if args.model == "resnet18" else "ResNet-50 (23.5M params)"
        return (
            make(num_classes=10, seed=1234),
            data,
            f"{n}, CIFAR stem, SGD(0.05, momentum 0.9, wd 5e-4)",
            "synthetic CIFAR-10-shaped (uint8 3x32x32), Dirichlet(0.5) non-IID shards, random-init weights",
        )
    if args.model == "vit_b16":
        from p2pfl_amd.data import ImageNetFederatedDM
        from p2pfl_amd.models.vit import ViT_B16

        ns = args.number_sub or 1
        data = ImageNetFederatedDM(sub_id=rank % ns, number_sub=ns, batch_size=args.batch, n_train=1024, seed=rank)
        return (
            ViT_B16(num_classes=1000, seed=1234),
            data,
            "ViT-B/16 (86.6M params, 197 tokens), AdamW(3e-4, wd 0.05)",
            "synthetic ImageNet-shaped (uint8 3x224x224, 1000 classes), random-init weights",
        )
    raise ValueError(args.model)


def learner_class(args):
    if args.impl == "fused" and args.model == "cnn":
        from p2pfl_amd.learning.fused_cnn import FusedCNNLearner

        return FusedCNNLearner
    from p2pfl_amd.learning.torch_learner import TorchLearner

    return TorchLearner


def _sync(dev: torch.device) -> None:
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


# ----------------------------------------------------------------------------
# launcher (parent process: never touches the GPU)
# ----------------------------------------------------------------------------
def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch(args, argv) -> int:
    """Start one worker process per GPU; return the first failing exit code."""
    import torch.distributed as dist

    n = args.gpus
    port = _free_port()
    # the job's c10d store lives here, so it survives any worker's death
    store = dist.TCPStore("127.0.0.1", port, n, True, wait_for_workers=False)  # noqa: F841
    job = uuid.uuid4().hex[:8]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), TORCHELASTIC_USE_AGENT_STORE="True",
                   TORCHELASTIC_RESTART_COUNT="0", P2PFL_JOB_ID=job)
        if os.environ.get("P2PFL_RCCL_SPLIT_HOSTS") == "1":
            # one-GPU rehearsal of the multi-rank RCCL path: RCCL rejects two
            # ranks on one device unless each looks like its own host, so the
            # ranks talk over RCCL's socket transport (loopback), not xGMI
            env.update(NCCL_HOSTID=f"p2pfl-{job}-r{r}", NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env, start_new_session=True))
    rc = 0
    deadline = time.monotonic() + args.watchdog + 60
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = bad[0]
                break
            if all(c == 0 for c in codes):
                break
            if time.monotonic() > deadline:
                print("[bench] launcher watchdog: workers did not finish", file=sys.stderr, flush=True)
                rc = 124
                break
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGTERM)
                except OSError:
                    pass
        for p in procs:
            try:
                p.wait(timeout=20)
            except subprocess.TimeoutExpired:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except OSError:
                    pass
    return rc


# ----------------------------------------------------------------------------
# worker: full-stack Node per rank, gossip over the xGMI transport
# ----------------------------------------------------------------------------
class _Env:
    def __init__(self) -> None:
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        if torch.cuda.is_available():
            idx = self.local % torch.cuda.device_count()
            torch.cuda.set_device(idx)
            self.device = torch.device("cuda", idx)
        else:
            self.device = torch.device("cpu")
        import torch.distributed as dist

        if self.world > 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("gloo", rank=self.rank, world_size=self.world)
            self.store = dist.distributed_c10d._get_default_store()
        else:
            self.store = dist.HashStore()

    def barrier(self) -> None:
        if self.world > 1:
            import torch.distributed as dist

            dist.barrier()

    def max(self, v: float) -> float:
        if self.world == 1:
            return v
        import torch.distributed as dist

        t = torch.tensor([v], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def sum(self, v: float) -> float:
        if self.world == 1:
            return v
        import torch.distributed as dist

        t = torch.tensor([v], dtype=torch.float64)
        dist.all_reduce(t)
        return float(t.item())

    def close(self) -> None:
        if self.world > 1:
            import torch.distributed as dist

            dist.destroy_process_group()


def run_gossip(args, env: _Env) -> dict:
    from p2pfl_amd.communication.xgmi import XgmiJob
    from p2pfl_amd.management.logger import logger
    from p2pfl_amd.node import Node
    from p2pfl_amd.settings import Settings

    N, W, K = env.world, args.warmup, args.steps
    Settings.LOG_LEVEL = os.environ.get("P2PFL_BENCH_LOG_LEVEL", "WARNING")
    Settings.TRAIN_SET_SIZE = N
    Settings.GOSSIP_MODELS_PER_ROUND = max(1, N - 1)
    Settings.TTL = 1
    Settings.WIRE_DTYPE = args.wire_dtype
    if os.environ.get("P2PFL_BENCH_NODE_STREAMS"):  # measurement knob: "0" / "1" / "auto"
        v = os.environ["P2PFL_BENCH_NODE_STREAMS"]
        Settings.NODE_STREAMS = v if v == "auto" else v == "1"
    # node addresses are machine-wide bus names: unique per job (self-launched
    # jobs carry P2PFL_JOB_ID, torchrun jobs their rendezvous port)
    job_id = os.environ.get("P2PFL_JOB_ID") or f"tr{os.environ.get('MASTER_PORT', '0')}-{os.getppid()}"
    job = XgmiJob(env.rank, N, env.store, device=env.device, backend=args.plane_backend, allow_fallback=args.allow_fallback,
                  prefix=f"p2pfl/{job_id}", job_id=job_id)
    torch.manual_seed(1234)  # identical init on every peer (the initiator's model wins anyway)
    model, data, desc, data_desc = build_config(args, env.rank)
    node = Node(model, data, protocol=job.protocol, learner=learner_class(args), device=env.device)
    marks = {}
    round_ends = {}

    def hook(state) -> None:
        r = state.round
        round_ends[r] = time.perf_counter()
        if r in (W, W + K):
            _sync(env.device)
            env.barrier()
            marks[r] = time.perf_counter()

    node.round_hooks.append(hook)
    node.start()
    try:
        # full mesh: rank i handshakes with every lower rank
        addrs = {}
        for r in range(N):
            a = env.store.get(f"{job.prefix}/addr/{r}")
            addrs[r] = a.decode() if isinstance(a, (bytes, bytearray)) else a
        for r in range(env.rank):
            if not node.connect(addrs[r]):
                raise RuntimeError(f"rank {env.rank} could not connect to rank {r}")
        t_end = time.monotonic() + 120
        while len(node.get_neighbors(only_direct=True)) < N - 1:
            if time.monotonic() > t_end:
                raise TimeoutError("full mesh did not form")
            time.sleep(0.01)
        plane = node._communication_protocol.plane
        if plane is not None and not plane.ready.wait(180):
            raise TimeoutError("data plane did not come up")
        if plane is not None and plane.failed:
            raise RuntimeError(plane.failed)
        # the backend the ranks actually agreed on (a fallback is reported, never hidden)
        backend_used = plane.backend_name if plane is not None else job.backend
        env.barrier()
        t_start = time.perf_counter()
        round_ends.setdefault(0, t_start)
        if W == 0:
            marks[0] = t_start
        if env.rank == 0:
            node.set_start_learning(rounds=W + K, epochs=args.epochs)
        t_end = time.monotonic() + args.watchdog
        while node._learning_thread is None:
            if time.monotonic() > t_end:
                raise TimeoutError("learning never started")
            time.sleep(0.001)
        if not node.wait_learning(timeout=args.watchdog):
            raise TimeoutError("learning did not finish")
        if W + K not in marks or W not in marks:
            raise RuntimeError(f"round marks missing: {sorted(marks)} (learning stopped early?)")
        elapsed = env.max(marks[W + K] - marks[W])
        # per-round phase breakdown from the tracer (this rank, timed rounds)
        sp = lambda name: [s for s in logger.tracer.spans(node.addr, name) if s.start >= marks[W]]  # noqa: E731
        ph = {k: sum(s.duration for s in sp(k)) / max(1, K) * 1e3 for k in ("evaluate", "fit", "wait_aggregation", "aggregate")}
        if os.environ.get("P2PFL_BENCH_SPANS"):
            tot: dict = {}
            for s in logger.tracer.spans(node.addr):
                if s.start >= marks[W]:
                    tot[s.name] = tot.get(s.name, 0.0) + s.duration
            print(f"[bench rank {env.rank}] all spans, ms per round: "
                  + ", ".join(f"{k} {v / max(1, K) * 1e3:.2f}" for k, v in sorted(tot.items(), key=lambda kv: -kv[1])),
                  file=sys.stderr, flush=True)
        if N > 1 or os.environ.get("P2PFL_BENCH_SPANS"):
            _print_round_breakdown(env.rank, node.addr, logger.tracer, round_ends, W, K)
        pushes = logger.tracer.counters(node.addr)
        stats = dict(plane.stats) if plane is not None else {}
        print(
            f"[bench rank {env.rank}] per-round (mean of {K}): " + ", ".join(f"{k} {v:.2f} ms" for k, v in ph.items())
            + f"; data plane: {stats.get('sent', 0)} sends / {stats.get('received', 0)} recvs / "
            f"{stats.get('groups', 0)} groups, {stats.get('nacked', 0)} declined"
            + "".join(f" [{k.split('/', 1)[1]}: {v}]" for k, v in sorted(stats.items()) if k.startswith("nacked/"))
            + f"; xgmi bytes sent {pushes.get('xgmi_bytes_sent', 0) / 1e6:.1f} MB",
            file=sys.stderr, flush=True,
        )
        from p2pfl_amd.ops import autotune

        if env.rank == 0 and autotune.choices():
            n_nat = sum(1 for v, _ in autotune.choices().values() if v.startswith("native"))
            print(f"[bench rank 0] kernel choice per shape (native vs library, ms): {n_nat}/{len(autotune.choices())} native\n"
                  + autotune.summary(), file=sys.stderr, flush=True)
        n_train = len(data.train_dataloader().dataset)
        n_val = len(data.val_dataloader().dataset)
        n_test = len(data.test_dataloader().dataset)
        per_peer_total = env.sum(n_train * args.epochs * K / elapsed)
        env.barrier()
    finally:
        node.stop()
    return {
        "elapsed": elapsed, "desc": desc, "data_desc": data_desc, "n_train": n_train, "n_val": n_val, "n_test": n_test,
        "total": per_peer_total, "parallelism": "gossip-p2p",
        "transport": f"xgmi/{backend_used}" + ("+split-hosts-rehearsal" if os.environ.get("NCCL_HOSTID") else ""),
    }


def _print_round_breakdown(rank, addr, tracer, round_ends, W, K) -> None:
    """Per-rank, per-round spans of the timed rounds (stderr): where a round's
    wall-clock went -- training, the pushes' propose->ack latency and group
    transfer times, bytes per link, the wait for the other peers' models, FedAvg."""
    rounds = [r for r in range(W + 1, W + K + 1) if r in round_ends and r - 1 in round_ends]
    spans = [s for s in tracer.spans(addr)]
    for r in rounds:
        t0, t1 = round_ends[r - 1], round_ends[r]
        inr = [s for s in spans if t0 <= s.start < t1]

        def tot(name):
            return sum(s.duration for s in inr if s.name == name) * 1e3

        acks = [s.duration * 1e3 for s in inr if s.name == "xgmi_ack"]
        groups = [s for s in inr if s.name == "xgmi_group"]
        gbytes = sum(int(s.attrs.get("nbytes", 0)) for s in groups)
        print(
            f"[bench rank {rank}] round {r}: wall {(t1 - t0) * 1e3:.2f} ms | fit {tot('fit'):.2f} (GPU epoch "
            f"{tot('train_epoch_gpu'):.2f}, between epochs {tot('inter_epoch_gpu'):.2f}) evaluate {tot('evaluate'):.2f} "
            f"wait_aggregation {tot('wait_aggregation'):.2f} aggregate {tot('aggregate'):.2f} | pushes: "
            f"ack {('%.3f' % (sum(acks) / len(acks))) if acks else '-'} ms mean over {len(acks)}, "
            f"{len(groups)} groups {sum(s.duration for s in groups) * 1e3:.2f} ms total "
            f"(max {max((s.duration for s in groups), default=0) * 1e3:.2f}), {gbytes / 1e6:.1f} MB moved",
            file=sys.stderr, flush=True,
        )
    links = {k.split("/", 1)[1]: v for k, v in tracer.counters(addr).items() if k.startswith("link_tx_bytes/")}
    if links:
        print(f"[bench rank {rank}] bytes sent per link over the run: "
              + ", ".join(f"->{p} {v / 1e6:.1f} MB" for p, v in sorted(links.items())), file=sys.stderr, flush=True)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3, help="timed federated rounds")
    ap.add_argument("--warmup", type=int, default=1, help="untimed federated rounds")
    ap.add_argument("--impl", choices=["fused", "torch"], default="fused")
    ap.add_argument("--model", choices=["cnn", "resnet18", "resnet50", "vit_b16"], default="cnn")
    ap.add_argument("--epochs", type=int, default=1)
    ap.add_argument("--number-sub", type=int, default=None, help="shards of the dataset (default per model)")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--wire-dtype", choices=["fp32", "bf16"], default="fp32", help="model arenas on the xGMI data plane")
    ap.add_argument("--watchdog", type=float, default=900, help="dump stacks and exit if the run hangs")
    ap.add_argument("--plane-backend", choices=["auto", "rccl", "gloo"], default="auto",
                    help="xGMI data-plane backend (auto: rccl on GPUs, gloo on CPUs)")
    ap.add_argument("--allow-fallback", action="store_true",
                    help="let the data plane degrade from RCCL to host-staged gloo instead of failing (the JSON "
                         "'transport' then says xgmi/gloo)")
    argv = sys.argv[1:]
    args = ap.parse_args(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch(args, argv))

    import faulthandler

    faulthandler.dump_traceback_later(args.watchdog, exit=True)
    env = _Env()
    if env.world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={env.world}")
    res = run_gossip(args, env)
    ms_per_round = res["elapsed"] / args.steps * 1e3
    total = res["total"]
    per_peer = total / env.world
    if env.rank == 0:
        print(
            json.dumps(
                {
                    "metric": "train samples/s (aggregate over peers); wall-clock per FedAvg round in ms_per_step",
                    "value": round(total, 1),
                    "unit": "samples/s",
                    "n_gpus": env.world,
                    "steps": args.steps,
                    "warmup": args.warmup,
                    "ms_per_step": round(ms_per_round, 3),
                    "samples_per_sec_per_peer": round(per_peer, 1),
                    "higher_is_better": True,
                    "scaling": "weak",
                    "vs_baseline": (round(per_peer / BASELINE_SAMPLES_PER_SEC_PER_PEER, 3) if args.model == "cnn" else None),
                    "dtype": "bf16" if env.device.type == "cuda" else "fp32",
                    "data": res["data_desc"],
                    "impl": args.impl if (args.model == "cnn" or args.impl != "fused") else "torch",
                    "transport": res["transport"],
                    "wire_dtype": args.wire_dtype,
                    "config": {
                        "model": res["desc"],
                        "global_batch": args.batch * env.world,
                        "seq_len": 197 if args.model == "vit_b16" else None,
                        "per_peer_round": f"{res['n_train']} train + {res['n_val']} val + {res['n_test']} test samples, "
                        f"{args.epochs} epoch",
                        "parallelism": res["parallelism"],
                    },
                }
            ),
            flush=True,
        )
    env.close()


if __name__ == "__main__":
    main()
