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


def poison_free_blocks(dev: torch.device, fill: bool = True) -> list:
    """Allocate (and, with ``fill``, NaN-fill) every free block of the caching allocator."""
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
            if fill:
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
    ap.add_argument("--hold-only", action="store_true", help="hold the free blocks but keep their content (no NaN)")
    a = ap.parse_args()
    if a.no_graphs:
        os.environ["P2PFL_STEP_GRAPHS"] = "0"
    from p2pfl_amd.data import Cifar10FederatedDM, MnistFederatedDM
    from p2pfl_amd.learning.torch_learner import TorchLearner

    dev = torch.device("cuda", 0)
    if a.model == "mlp":
        from p2pfl_amd.models import MLP

        model, data = MLP(seed=1), MnistFederatedDM(sub_id=0, number_sub=20)
    elif a.model == "vit_tiny":
        from p2pfl_amd.models.vit import ViT_Tiny

        model, data = ViT_Tiny(seed=0), Cifar10FederatedDM(sub_id=0, number_sub=40)
    else:
        from p2pfl_amd.models.resnet import ResNet18, ResNet50

        model = (ResNet50 if a.model == "resnet50" else ResNet18)(seed=1234)
        data = Cifar10FederatedDM(sub_id=0, number_sub=64, partitioner="dirichlet", alpha=0.5)
    ln = TorchLearner(model, data, "poison", 1, device=dev)
    keep = []
    for i in range(a.fits):
        ln.fit()
        torch.cuda.synchronize(dev)
        flat = ln.get_parameters().flat
        bad = int((~torch.isfinite(flat)).sum())
        print(f"fit {i}: non-finite parameters {bad} of {flat.numel()}; graph={ln._step_graph is not None}", flush=True)
        if bad:
            names = ln.arena.layout.names
            per = [(n, int((~torch.isfinite(t)).sum()), t.numel()) for n, t in ln.get_parameters().items()]
            first = [p for p in per if p[1]]
            print(f"non-finite tensors: {len(first)} of {len(per)}; first ones in layout order:", flush=True)
            for n, k, m in first[:12]:
                print(f"   {n}: {k}/{m}", flush=True)
            print(f"   last: {first[-1][0]}", flush=True)
            sys.exit(2)
        if (a.poison or a.hold_only) and i == 0:
            keep = poison_free_blocks(dev, fill=not a.hold_only)
            print(f"poisoned {sum(t.numel() for t in keep) * 4 / 2**20:.1f} MiB of free cached blocks in {len(keep)} tensors",
                  flush=True)
    print("all fits finite", flush=True)


if __name__ == "__main__":
    main()
