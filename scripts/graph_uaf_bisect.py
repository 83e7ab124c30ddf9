"""Find the freed block a captured training-step graph still reads.

``scripts/graph_poison.py`` showed that filling every free block of the
caching allocator with NaN after the step graph was captured makes the next
graph-replayed fit non-finite (ResNet-50), while the eager path stays finite.
This script names the block: it holds every free block (as "poison"
tensors), then bisects over them -- NaN in one half, the stale content the
blocks held when they were taken in the other,
model and optimizer state restored before every trial -- down to one block,
and looks its address up in the allocator's history (who allocated and freed
that memory before the poison took it).

    python scripts/graph_uaf_bisect.py [--model resnet50]
"""

from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    a = ap.parse_args()
    torch.cuda.memory._record_memory_history(max_entries=500000, stacks="python")
    from p2pfl_amd.data import Cifar10FederatedDM
    from p2pfl_amd.learning.torch_learner import TorchLearner
    from p2pfl_amd.models.resnet import ResNet18, ResNet50
    from scripts.graph_poison import poison_free_blocks

    dev = torch.device("cuda", 0)
    model = (ResNet50 if a.model == "resnet50" else ResNet18)(seed=1234)
    ln = TorchLearner(model, Cifar10FederatedDM(sub_id=0, number_sub=64, partitioner="dirichlet", alpha=0.5),
                      "bisect", 1, device=dev)
    ln.fit()  # captures the step graph
    torch.cuda.synchronize(dev)
    opt = ln._mt_opt
    state = [ln.arena.flat, ln.arena.shadow] + (opt.state_tensors() if opt is not None else [])
    state = [t for t in state if t is not None]
    ints = getattr(ln.arena, "_int_buffers", {})
    saved = [t.clone() for t in state]
    saved_ints = {k: v.clone() for k, v in ints.items()}
    snap = torch.cuda.memory._snapshot()
    poison = poison_free_blocks(dev, fill=False)
    orig = [t.clone() for t in poison]  # what the freed blocks held when the poison took them
    print(f"holding {len(poison)} free blocks ({sum(t.numel() for t in poison) * 4 / 2**20:.1f} MiB)", flush=True)

    def trial(nan_set) -> bool:
        for dst, src in zip(state, saved):
            dst.copy_(src)
        for k, v in saved_ints.items():
            ints[k].copy_(v)
        for i, t in enumerate(poison):
            if i in nan_set:
                t.fill_(float("nan"))
            else:
                t.copy_(orig[i])
        torch.cuda.synchronize(dev)
        ln.fit()
        torch.cuda.synchronize(dev)
        return bool((~torch.isfinite(ln.arena.flat)).any())

    cand = list(range(len(poison)))
    if not trial(set(cand)):
        print("no NaN with every free block poisoned: nothing to bisect", flush=True)
        return
    if trial(set()):
        print("NaN with every held block restored to its stale content: not a freed-block read", flush=True)
        return
    while len(cand) > 1:
        half = cand[: len(cand) // 2]
        if trial(set(half)):
            cand = half
        else:
            rest = cand[len(cand) // 2:]
            if trial(set(rest)):
                cand = rest
            else:
                print(f"NaN needs blocks from both halves of {len(cand)}; stopping", flush=True)
                break
    for i in cand[:4]:
        t = poison[i]
        lo, hi = t.data_ptr(), t.data_ptr() + t.numel() * 4
        print(f"culprit block: [{lo:#x}, {hi:#x}) {hi - lo} bytes", flush=True)
        # allocator history of that address range before the poison took it
        events = []
        for trace in snap.get("device_traces", []):
            for ev in trace:
                addr, size = ev.get("addr", 0), ev.get("size", 0)
                if addr < hi and addr + size > lo and ev.get("action") in ("alloc", "free_requested", "free_completed"):
                    events.append(ev)
        print(f"  {len(events)} allocator events touched it before the poison; the last ones:", flush=True)
        for ev in events[-6:]:
            frames = [f"{f.get('filename', '?').split('/')[-1]}:{f.get('line', '?')}:{f.get('name', '?')}"
                      for f in ev.get("frames", []) if "torch/" not in f.get("filename", "")][:8]
            print(f"  {ev.get('action')} addr={ev.get('addr', 0):#x} size={ev.get('size')} stream={ev.get('stream')}"
                  f"\n      " + "\n      ".join(frames), flush=True)


if __name__ == "__main__":
    main()
