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


from p2pfl_amd.utils.alloc_probe import poison_free_blocks  # noqa: E402,F401  (re-exported for graph_uaf_bisect)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--poison", action="store_true")
    ap.add_argument("--fits", type=int, default=3)
    ap.add_argument("--hold-only", action="store_true", help="hold the free blocks but keep their content (no NaN)")
    ap.add_argument("--trace-steps", action="store_true")
    ap.add_argument("--fresh", choices=("nan", "zero", "one"), default=None,
                    help="before fit 1: hold the free blocks, then fill one big new block with this value and free it, "
                         "so fit 1's new allocations come from memory of known content")
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
    if a.trace_steps:
        # name the first step of the second fit whose loss or weights turn non-finite
        from p2pfl_amd.learning.step_graph import TrainStepGraph

        state = {"fit": 0, "step": 0, "reported": False}
        orig_run = TrainStepGraph.run

        def run(self, idx):
            loss = orig_run(self, idx)
            if state["fit"] == 1 and not state["reported"]:
                torch.cuda.synchronize(dev)
                lf = bool(torch.isfinite(loss).all())
                wf = bool(torch.isfinite(ln.arena.flat).all())
                if state["step"] < 3 or not (lf and wf):
                    print(f"   replay {state['step']}: loss {float(loss):.4f} finite={lf} weights finite={wf}", flush=True)
                if not (lf and wf):
                    state["reported"] = True
            state["step"] += 1
            return loss

        TrainStepGraph.run = run
    keep = []
    for i in range(a.fits):
        ln.fit()
        torch.cuda.synchronize(dev)
        flat = ln.get_parameters().flat
        bad = int((~torch.isfinite(flat)).sum())
        sg = ln._step_graph
        print(f"fit {i}: non-finite parameters {bad} of {flat.numel()}; graph={sg is not None} "
              f"graph_id={id(sg.graph) if sg is not None and sg.graph is not None else None}", flush=True)
        if bad:
            names = ln.arena.layout.names
            per = [(n, int((~torch.isfinite(t)).sum()), t.numel()) for n, t in ln.get_parameters().items()]
            first = [p for p in per if p[1]]
            print(f"non-finite tensors: {len(first)} of {len(per)}; first ones in layout order:", flush=True)
            for n, k, m in first[:12]:
                print(f"   {n}: {k}/{m}", flush=True)
            print(f"   last: {first[-1][0]}", flush=True)
            sys.exit(2)
        if a.fresh and i == 0:
            keep = poison_free_blocks(dev, fill=False)
            free_b = torch.cuda.mem_get_info(dev)[0]
            big = torch.empty(int(free_b * 0.5) // 4, dtype=torch.float32, device=dev)
            big.fill_({"nan": float("nan"), "zero": 0.0, "one": 1.0}[a.fresh])
            torch.cuda.synchronize(dev)
            print(f"held {len(keep)} free blocks; {big.numel() * 4 / 2**30:.1f} GiB of fresh memory filled with "
                  f"{a.fresh} and returned to the cache", flush=True)
            del big
        if a.trace_steps:
            state["fit"], state["step"] = i + 1, 0
            print(f"   after fit {i}: weights finite={bool(torch.isfinite(ln.arena.flat).all())}", flush=True)
        if (a.poison or a.hold_only) and i == 0:
            keep = poison_free_blocks(dev, fill=not a.hold_only)
            print(f"poisoned {sum(t.numel() for t in keep) * 4 / 2**20:.1f} MiB of free cached blocks in {len(keep)} tensors",
                  flush=True)
    print("all fits finite", flush=True)


if __name__ == "__main__":
    main()
