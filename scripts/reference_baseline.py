"""The measured reference-equivalent baseline of BASELINE.md: one peer's FedAvg round
done the way p2pfl v0.3's LightningLearner does it, minus Lightning itself.

    python scripts/reference_baseline.py [--steps 3] [--warmup 1] [--model cnn]

fp32 eager PyTorch, the double forward of every evaluation step
(/root/reference/p2pfl/learning/pytorch/mnist_examples/models/cnn.py:103-104),
Adam re-created per fit, pickle encode / decode of the whole model
(lightning_learner.py:123-136) and the per-layer FedAvg loop (fedavg.py:49-58),
on one GPU (or the CPU).  Same per-peer shard and model as ``bench.py``; prints one
JSON line with ms per round and train samples/s.  The reference's control-plane
sleeps (>= 2 s per round with default Settings) are NOT included, which makes this
baseline strictly faster than the reference itself.  (Round 1 measured it as
``bench.py --impl reference``: 99.6 ms / round, 27,120.7 samples/s on one MI355X.)
"""

from __future__ import annotations

import argparse
import json
import os
import pickle
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import bench  # noqa: E402


class ReferenceEquivalentLearner:
    """What p2pfl's LightningLearner does per round, minus Lightning itself."""

    def __init__(self, model, data, device):
        self.model = model.to(device)
        self.data = data.to(device)
        self.device = device
        self._keys = list(self.model.state_dict().keys())

    def evaluate(self, loader) -> float:
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

    def fit(self) -> None:
        self.model.train()
        opt = torch.optim.Adam(self.model.parameters(), lr=1e-3)  # re-created per fit (reference quirk Q23)
        for x, y in self.data.train_dataloader():
            opt.zero_grad()
            loss = torch.nn.functional.cross_entropy(self.model(x), y)
            loss.backward()
            opt.step()
        self.evaluate(self.data.val_dataloader())

    def get_parameters(self):
        # reference encode: .cpu().numpy() + pickle; decode: pickle.loads + torch.tensor (own data, trusted)
        blob = pickle.dumps([v.cpu().numpy() for v in self.model.state_dict().values()])
        arrays = pickle.loads(blob)
        return [torch.tensor(a, device=self.device) for a in arrays]

    def set_parameters(self, params) -> None:
        self.model.load_state_dict(dict(zip(self._keys, params)))


def reference_round(learner: ReferenceEquivalentLearner, weight: float) -> float:
    t0 = time.perf_counter()
    learner.evaluate(learner.data.test_dataloader())
    learner.fit()
    params = learner.get_parameters()
    accum = [torch.zeros_like(p) for p in params]
    for model in [params]:  # per-layer FedAvg loop (reference fedavg.py:49-58), one peer
        for i, layer in enumerate(model):
            accum[i] = accum[i] + layer * weight
    learner.set_parameters([a / weight for a in accum])
    if learner.device.type == "cuda":
        torch.cuda.synchronize(learner.device)
    return time.perf_counter() - t0


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--model", choices=["cnn", "resnet18", "resnet50", "vit_b16"], default="cnn")
    ap.add_argument("--number-sub", type=int, default=None)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--epochs", type=int, default=1)
    args = ap.parse_args()
    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    torch.manual_seed(1234)
    model, data, desc, data_desc = bench.build_config(args, 0)
    learner = ReferenceEquivalentLearner(model, data, dev)
    weight = float(len(data.train_dataloader().dataset))
    for i in range(args.warmup):
        print(f"[reference] warmup round {i}: {reference_round(learner, weight) * 1e3:.2f} ms", file=sys.stderr, flush=True)
    t = sum(reference_round(learner, weight) for _ in range(args.steps))
    n_train = len(data.train_dataloader().dataset)
    print(json.dumps({"metric": "reference-equivalent FedAvg round", "ms_per_round": round(t / args.steps * 1e3, 3),
                      "train_samples_per_sec": round(n_train * args.steps / t, 1), "model": desc, "data": data_desc,
                      "device": str(dev), "dtype": "fp32"}), flush=True)


if __name__ == "__main__":
    main()
