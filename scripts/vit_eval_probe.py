"""ViT-B/16 evaluation passes of the bench round in isolation: device ms per test pass
(1000 images: 3 captured 256-image graphs + a 232-image tail) and per validation pass,
next to one training epoch, through the same TorchLearner the bench drives.

    python scripts/vit_eval_probe.py [--reps 5]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--no-fit", action="store_true")
    ap.add_argument("--no-val", action="store_true", help="test passes only (a profile window of test passes)")
    args = ap.parse_args()
    from p2pfl_amd.data import ImageNetFederatedDM
    from p2pfl_amd.learning.torch_learner import TorchLearner
    from p2pfl_amd.models.vit import ViT_B16

    dev = torch.device("cuda")
    data = ImageNetFederatedDM(batch_size=32, n_train=1024, seed=0)
    lr = TorchLearner(ViT_B16(num_classes=1000, seed=1234), data, "probe", 1, device=dev)

    def timed(fn):
        torch.cuda.synchronize()
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) * 1e3

    res = {}
    if not args.no_fit:
        lr.fit()
        res["fit_ms"] = [round(timed(lr.fit), 2) for _ in range(2)]
    lr.evaluate()
    res["test_ms"] = [round(timed(lr.evaluate), 2) for _ in range(args.reps)]
    if not args.no_val:
        lr.validate()
        res["val_ms"] = [round(timed(lr.validate), 2) for _ in range(args.reps)]
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
