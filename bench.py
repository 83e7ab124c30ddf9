"""Headline benchmark: MNIST-CNN FedAvg rounds, one federated peer per GPU.

Metric (BASELINE.json): wall-clock per round + samples/s per peer, MNIST-CNN
FedAvg at 1/2/4/8 peers.  ``value`` is the whole-job aggregate training
throughput (train samples/s summed over peers); ``ms_per_step`` is the
wall-clock of one federated round.

Per-peer round (weak scaling -- fixed per-peer work as N grows), matching the
reference example ``p2pfl/examples/mnist.py`` shard (``MnistFederatedDM(sub_id,
number_sub=20)``): 2,700 train / 300 val / 500 test MNIST-shaped samples,
batch 32, the reference CNN (6.5 M params), Adam lr 1e-3 re-created per round,
1 local epoch:

    evaluate(test) -> fit(1 epoch + val) -> FedAvg over all peers (RCCL) -> load

Implementations (``--impl``):
  fused      hand-written HIP/CDNA4 CNN step (MFMA GEMMs, fused epilogues,
             fused Adam), HIP-graph-captured; flat-arena FedAvg   [default]
  torch      PyTorch-ROCm autograd (bf16 autocast) + fused arena Adam kernel
  reference  reference-equivalent path: fp32 eager PyTorch, torch.optim.Adam,
             double-forward eval, pickle encode/decode of the model and a
             per-layer FedAvg loop (what p2pfl's Lightning learner executes),
             used to measure the baseline on the same MI355X.

Other BASELINE.json configurations (``--model``, PyTorch-ROCm path with the
fused arena optimiser and, for ViT, the fused LayerNorm/GELU/xent kernels):
  resnet18   CIFAR-10-shaped, non-IID Dirichlet(0.5) shards, SGD-momentum (config 3)
  resnet50   CIFAR-10-shaped, Dirichlet shards (config 5's model)
  vit_b16    ImageNet-shaped 224x224 (197 tokens), AdamW (config 4)

Run:  python bench.py --gpus 1 --steps 3 --warmup 1
      python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""

from __future__ import annotations

import argparse
import json
import os
import pickle
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

from p2pfl_amd.data import MnistFederatedDM  # noqa: E402
from p2pfl_amd.models import CNN  # noqa: E402
from p2pfl_amd.parallel import CollectiveFedAvg, init_distributed  # noqa: E402
from p2pfl_amd.parallel.rounds import FederatedRoundRunner  # noqa: E402

# Reference-equivalent baseline, measured (not published -- the reference
# publishes no timing): `python bench.py --impl reference` on one MI355X,
# 99.6 ms per round = 27,120.7 train samples/s per peer.
# vs_baseline compares per-peer throughput (value / n_gpus) with it.
BASELINE_SAMPLES_PER_SEC_PER_PEER = 27120.7


class ReferenceEquivalentLearner:
    """What p2pfl's LightningLearner does per round, minus Lightning itself."""

    def __init__(self, model, data, device):
        self.model = model.to(device)
        self.data = data.to(device)
        self.device = device

    def get_num_samples(self):
        return len(self.data.train_dataloader().dataset), len(self.data.test_dataloader().dataset)

    def _eval(self, loader):
        self.model.eval()
        tot, n = 0.0, 0
        with torch.no_grad():
            for x, y in loader:
                logits = self.model(x)
                loss = torch.nn.functional.cross_entropy(self.model(x), y)  # double forward (reference cnn.py:103-104)
                acc = (logits.argmax(1) == y).float().mean()
                tot += float(loss) * len(y) + 0 * float(acc)
                n += len(y)
        return tot / max(n, 1)

    def evaluate(self):
        return {"test_loss": self._eval(self.data.test_dataloader())}

    def fit(self):
        self.model.train()
        opt = torch.optim.Adam(self.model.parameters(), lr=1e-3)
        for x, y in self.data.train_dataloader():
            opt.zero_grad()
            loss = torch.nn.functional.cross_entropy(self.model(x), y)
            loss.backward()
            opt.step()
        self._eval(self.data.val_dataloader())

    def get_parameters(self):
        # reference encode: .cpu().numpy() + pickle; decode: pickle.loads + torch.tensor
        blob = pickle.dumps([v.cpu().numpy() for v in self.model.state_dict().values()])
        arrays = pickle.loads(blob)
        self._keys = list(self.model.state_dict().keys())
        return [torch.tensor(a, device=self.device) for a in arrays]

    def set_parameters(self, params):
        self.model.load_state_dict(dict(zip(self._keys, params)))


def reference_round(learner, env, weight, total):
    import torch.distributed as dist

    t0 = time.perf_counter()
    learner.evaluate()
    learner.fit()
    params = learner.get_parameters()
    # per-layer FedAvg over all peers' models (reference fedavg.py:49-58)
    gathered = [params]
    if env.world_size > 1:
        gathered = []
        for r in range(env.world_size):
            gathered.append([p.clone() for p in params])
        for i, p in enumerate(params):
            outs = [torch.empty_like(p) for _ in range(env.world_size)]
            dist.all_gather(outs, p)
            for r in range(env.world_size):
                gathered[r][i] = outs[r]
    accum = [torch.zeros_like(p) for p in params]
    for model in gathered:
        for i, layer in enumerate(model):
            accum[i] = accum[i] + layer * weight
    accum = [a / (weight * len(gathered)) for a in accum]
    learner.set_parameters(accum)
    _sync()
    return time.perf_counter() - t0


def build_config(args, env):
    """(model, data module, model description, data description) for ``--model``."""
    sub = env.rank
    if args.model == "cnn":
        ns = args.number_sub or 20
        data = MnistFederatedDM(sub_id=sub % ns, number_sub=ns, batch_size=args.batch)
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
        data = Cifar10FederatedDM(sub_id=sub % ns, number_sub=ns, batch_size=args.batch, partitioner="dirichlet", alpha=0.5)
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
        data = ImageNetFederatedDM(sub_id=sub % ns, number_sub=ns, batch_size=args.batch, n_train=1024, seed=sub)
        return (
            ViT_B16(num_classes=1000, seed=1234),
            data,
            "ViT-B/16 (86.6M params, 197 tokens), AdamW(3e-4, wd 0.05)",
            "synthetic ImageNet-shaped (uint8 3x224x224, 1000 classes), random-init weights",
        )
    raise ValueError(args.model)


def _sync() -> None:
    if torch.cuda.is_available():
        torch.cuda.synchronize()


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3, help="timed federated rounds")
    ap.add_argument("--warmup", type=int, default=1, help="untimed federated rounds")
    ap.add_argument("--impl", choices=["fused", "torch", "reference"], default="fused")
    ap.add_argument("--model", choices=["cnn", "resnet18", "resnet50", "vit_b16"], default="cnn")
    ap.add_argument("--epochs", type=int, default=1)
    ap.add_argument("--number-sub", type=int, default=None, help="shards of the dataset (default per model)")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--watchdog", type=float, default=900, help="dump stacks and exit if the run hangs")
    args = ap.parse_args()
    import faulthandler

    faulthandler.dump_traceback_later(args.watchdog, exit=True)

    env = init_distributed()
    assert env.world_size == args.gpus, f"--gpus {args.gpus} but WORLD_SIZE={env.world_size}"
    dev = env.device
    torch.manual_seed(1234)  # identical init on every peer (the initiator's model)
    model, data, desc, data_desc = build_config(args, env)
    fed = CollectiveFedAvg(env)

    if args.impl == "reference":
        learner = ReferenceEquivalentLearner(model, data, dev)
        weight = float(learner.get_num_samples()[0])
        total = fed.total_weight(weight)
        run = lambda: reference_round(learner, env, weight, total)  # noqa: E731
    else:
        if args.impl == "fused" and args.model == "cnn":
            from p2pfl_amd.learning.fused_cnn import FusedCNNLearner as L
        else:
            from p2pfl_amd.learning.torch_learner import TorchLearner as L
        learner = L(model, data, f"peer{env.rank}", args.epochs, device=dev)
        runner = FederatedRoundRunner(learner, fed, name=f"peer{env.rank}")
        run = lambda: runner.run_round().seconds  # noqa: E731

    for i in range(args.warmup):
        t = run()
        print(f"[bench rank {env.rank}] warmup round {i}: {t * 1e3:.2f} ms", file=sys.stderr, flush=True)
    fed.barrier()
    _sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run()
    _sync()
    fed.barrier()
    elapsed = fed.max_over_ranks(time.perf_counter() - t0)

    if args.impl != "reference" and runner.history:
        h = runner.history[-args.steps:]
        k = len(h)
        print(
            f"[bench rank {env.rank}] per-round phases (mean of {k}): evaluate {sum(x.eval_s for x in h) / k * 1e3:.2f} ms, "
            f"fit {sum(x.fit_s for x in h) / k * 1e3:.2f} ms, fedavg+load (+overlapped val) {sum(x.agg_s for x in h) / k * 1e3:.2f} ms",
            file=sys.stderr,
            flush=True,
        )
    n_train = len(data.train_dataloader().dataset)
    ms_per_round = elapsed / args.steps * 1e3
    per_peer = n_train * args.epochs * args.steps / elapsed
    total = per_peer * env.world_size
    if env.is_main:
        base = BASELINE_SAMPLES_PER_SEC_PER_PEER
        print(
            json.dumps(
                {
                    "metric": "train samples/s (aggregate over peers); wall-clock per FedAvg round in ms_per_step",
                    "value": round(total, 1),
                    "unit": "samples/s",
                    "n_gpus": env.world_size,
                    "steps": args.steps,
                    "warmup": args.warmup,
                    "ms_per_step": round(ms_per_round, 3),
                    "samples_per_sec_per_peer": round(per_peer, 1),
                    "higher_is_better": True,
                    "scaling": "weak",
                    "vs_baseline": (round(per_peer / base, 3) if (base and args.model == "cnn") else None),
                    "dtype": "bf16" if (args.impl != "reference" and dev.type == "cuda") else "fp32",
                    "data": data_desc,
                    "impl": args.impl if (args.model == "cnn" or args.impl != "fused") else "torch",
                    "config": {
                        "model": desc,
                        "global_batch": args.batch * env.world_size,
                        "seq_len": 197 if args.model == "vit_b16" else None,
                        "per_peer_round": f"{n_train} train + {len(data.val_dataloader().dataset)} val + "
                        f"{len(data.test_dataloader().dataset)} test samples, {args.epochs} epoch",
                        "parallelism": f"fedavg-dp{env.world_size}",
                    },
                }
            ),
            flush=True,
        )


if __name__ == "__main__":
    main()
