"""Does a captured training step graph read memory it does not own?

Trains a TorchLearner (ResNet, HIP-graph step replay) for one fit, then fills
every free block of PyTorch's caching allocator with NaN (and keeps it
allocated), then fits again.  A graph whose kernels still reference memory
that was freed after the capture (a use-after-free that only shows up when
something else reuses those blocks, e.g. a profiler's buffers) now reads NaN.

    python scripts/graph_poison.py [--model resnet50|resnet18] [--no-graphs] [--poison]
"""

from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def poison_free_blocks(dev: torch.device) -> list:
    """Allocate (and NaN-fill) every free block of the caching allocator."""
    keep = []
    sizes = [1 << s for s in range(30, 9, -1)]
    for sz in sizes:
        while True:
            free_cached = torch.cuda.memory_reserved(dev) - torch.cuda.memory_allocated(dev)
            if free_cached < sz:
                break
            before = torch.cuda.memory_reserved(dev)
            t = torch.empty(sz // 4, dtype=torch.float32, device=dev)
            if torch.cuda.memory_reserved(dev) > before:  # new segment: not a freed block
                del t
                break
            t.fill_(float("nan"))
            keep.append(t)
    torch.cuda.synchronize(dev)
    return keep


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--poison", action="store_true")
    ap.add_argument("--fits", type=int, default=3)
    a = ap.parse_args()
    if a.no_graphs:
        os.environ["P2PFL_STEP_GRAPHS"] = "0"
    from p2pfl_amd.data import Cifar10FederatedDM
    from p2pfl_amd.learning.torch_learner import TorchLearner
    from p2pfl_amd.models.resnet import ResNet18, ResNet50

    dev = torch.device("cuda", 0)
    net = ResNet50 if a.model == "resnet50" else ResNet18
    ln = TorchLearner(net(seed=1234), Cifar10FederatedDM(sub_id=0, number_sub=64, partitioner="dirichlet", alpha=0.5),
                      "poison", 1, device=dev)
    keep = []
    for i in range(a.fits):
        ln.fit()
        torch.cuda.synchronize(dev)
        flat = ln.get_parameters().flat
        bad = int((~torch.isfinite(flat)).sum())
        print(f"fit {i}: non-finite parameters {bad} of {flat.numel()}; graph={ln._step_graph is not None}", flush=True)
        if bad:
            sys.exit(2)
        if a.poison and i == 0:
            keep = poison_free_blocks(dev)
            print(f"poisoned {sum(t.numel() for t in keep) * 4 / 2**20:.1f} MiB of free cached blocks in {len(keep)} tensors",
                  flush=True)
    print("all fits finite", flush=True)


if __name__ == "__main__":
    main()
