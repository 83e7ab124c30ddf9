"""Host cost of replaying a captured HIP graph (hipGraphLaunch) vs its node count.

The fused CNN's training epoch is one graph of ~660 kernel nodes, and
rocprofv3 --hip-trace shows each replay's hipGraphLaunch holding the host for
~6.4 ms (profiles/r5_cnn_gaps.md).  This separates the two explanations:
  * per-node host work inside the launch: the time scales with the node count
    and does not depend on whether the device is busy;
  * back-pressure from a full hardware queue: the launch returns quickly while
    the device idles, slowly when a long kernel is queued ahead of it.

    python scripts/graph_launch_probe.py
"""

from __future__ import annotations

import time

import torch


def main() -> None:
    dev = torch.device("cuda")
    x = torch.zeros(256, device=dev)
    s = torch.cuda.Stream()
    for n in (50, 200, 660, 2000):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            for _ in range(3):
                x.add_(1.0)
            torch.cuda.synchronize()
            with torch.cuda.graph(g, stream=s):
                for _ in range(n):
                    x.add_(1.0)
        torch.cuda.synchronize()
        res = {}
        for mode in ("idle", "busy"):
            ts = []
            for _ in range(5):
                torch.cuda.synchronize()
                if mode == "busy":
                    torch.cuda._sleep(int(2e8))  # ~100 ms of device work queued ahead
                t0 = time.perf_counter()
                g.replay()
                ts.append(time.perf_counter() - t0)
                torch.cuda.synchronize()
            res[mode] = sorted(ts)[len(ts) // 2] * 1e6
        # device time of one replay
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        b.synchronize()
        print(f"{n} nodes: hipGraphLaunch host {res['idle']:.0f} us (device idle), {res['busy']:.0f} us (device busy); "
              f"{res['idle'] / n:.1f} us/node; device time {a.elapsed_time(b) * 1e3:.0f} us", flush=True)


def cnn_epoch(steps: int = 94, B: int = 32) -> None:
    """The same measurement on the fused CNN's real training epoch graph."""
    from p2pfl_amd.learning.fused_cnn import FusedCNNEngine
    from p2pfl_amd.models import CNN

    dev = torch.device("cuda")
    torch.manual_seed(0)
    eng = FusedCNNEngine(CNN(seed=0).to(dev), device=dev, lr=1e-3)
    n = steps * B
    x = torch.randint(0, 256, (n, 784), dtype=torch.uint8, device=dev)
    y = torch.randint(0, 10, (n,), device=dev)
    perm = torch.randperm(n, device=dev)
    stats = torch.zeros((steps, 4), device=dev)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for j in range(2):
            eng.train_step_async(x, y, perm[j * B:(j + 1) * B], B, stats[j], j + 1)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for j in range(steps):
            eng.train_step_async(x, y, perm[j * B:(j + 1) * B], B, stats[j], j + 1)
    torch.cuda.synchronize()
    res = {}
    for mode in ("idle", "busy", "back-to-back"):
        ts = []
        for _ in range(5):
            torch.cuda.synchronize()
            if mode == "busy":
                torch.cuda._sleep(int(2e8))
            if mode == "back-to-back":
                g.replay()
            t0 = time.perf_counter()
            g.replay()
            ts.append(time.perf_counter() - t0)
            torch.cuda.synchronize()
        res[mode] = sorted(ts)[len(ts) // 2] * 1e6
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    g.replay()
    b.record()
    b.synchronize()
    print(f"CNN epoch graph ({steps} steps x 7 kernels): hipGraphLaunch host {res['idle']:.0f} us (device idle), "
          f"{res['busy']:.0f} us (device busy), {res['back-to-back']:.0f} us (second of two back-to-back replays); "
          f"device time {a.elapsed_time(b) * 1e3:.0f} us", flush=True)
    # sustained: 150 replays back to back (about a second of load, as in a benchmark
    # run), device time per replay over consecutive windows -- clock settling shows here
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(151)]
    with torch.cuda.stream(s):
        evs[0].record(s)
        for i in range(150):
            g.replay()
            evs[i + 1].record(s)
    torch.cuda.synchronize()
    per = [evs[i].elapsed_time(evs[i + 1]) * 1e3 for i in range(150)]
    win = [sum(per[i:i + 30]) / 30 for i in range(0, 150, 30)]
    print("sustained replays, mean device us per epoch over windows of 30: " + ", ".join(f"{w:.0f}" for w in win), flush=True)


if __name__ == "__main__":
    import os
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    main()
    cnn_epoch()
