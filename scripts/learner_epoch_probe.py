"""Device time of the fused CNN learner's epoch (its own captured graph, as bench.py
replays it) against the same engine's steps captured by hand (graph_launch_probe's
cnn_epoch): isolates what the learner path adds per step.

    python scripts/learner_epoch_probe.py
"""

from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from p2pfl_amd.data import MnistFederatedDM  # noqa: E402
from p2pfl_amd.learning.fused_cnn import FusedCNNLearner  # noqa: E402
from p2pfl_amd.models import CNN  # noqa: E402


def main() -> None:
    dev = torch.device("cuda")
    data = MnistFederatedDM(sub_id=0, number_sub=20, batch_size=32)
    lrn = FusedCNNLearner(CNN(seed=0), data, "probe", 1, device=dev)
    loader = data.train_dataloader()
    steps = -(-len(loader.dataset) // loader.batch_size)
    for _ in range(3):  # captures, autotune, warm-up
        lrn.fit()
    lrn.drain()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    # (1) the learner's epoch graph alone, replayed on the current stream
    g = lrn._graphs["train"]
    with torch.cuda.stream(torch.cuda.Stream()):
        cur = torch.cuda.current_stream()
        for _ in range(3):
            g.graph.replay()
        a.record(cur)
        for _ in range(20):
            g.graph.replay()
        b.record(cur)
    torch.cuda.synchronize()
    us = a.elapsed_time(b) * 1e3 / 20
    print(f"learner epoch graph alone: {us:.0f} us per epoch of {steps} steps = {us / steps:.1f} us/step", flush=True)
    # (1b) the epoch as fit() enqueues it, without the validation pass: optimizer
    # reset, batch order copy, replay, stats readback -- on the learner's stream
    def epoch_only():
        with lrn._on_stream():
            lrn.engine.reset_optimizer()
            stats = lrn._run("train", loader, True, loader.permutation(host=True))
            lrn._readback(stats)

    def epoch_and_validation():
        epoch_only()
        with lrn._on_stream():
            lrn._validate_async()

    def replay_on_stream():
        with lrn._on_stream():
            lrn._run("train", loader, True, None)

    def reset_replay():
        with lrn._on_stream():
            lrn.engine.reset_optimizer()
            lrn._run("train", loader, True, None)

    def reset_perm_replay():
        with lrn._on_stream():
            lrn.engine.reset_optimizer()
            lrn._run("train", loader, True, loader.permutation(host=True))

    def reset_devperm_replay():
        with lrn._on_stream():
            lrn.engine.reset_optimizer()
            lrn._run("train", loader, True, loader.permutation())

    cs = lrn._stream_for_block()
    legacy = torch.cuda.default_stream()
    side = torch.cuda.Stream()

    def on_cs_no_handoff():
        with torch.cuda.stream(cs):
            g.graph.replay()

    def on_cs_handoff_legacy():
        cs.wait_stream(legacy)
        with torch.cuda.stream(cs):
            g.graph.replay()
        legacy.wait_stream(cs)

    def on_cs_handoff_side():
        cs.wait_stream(side)
        with torch.cuda.stream(cs):
            g.graph.replay()
        side.wait_stream(cs)

    def on_legacy():
        with torch.cuda.stream(legacy):
            g.graph.replay()

    import time

    host = []
    for _ in range(5):  # host time of each hand-off call right after an enqueued replay
        t0 = time.perf_counter()
        cs.wait_stream(legacy)
        t1 = time.perf_counter()
        with torch.cuda.stream(cs):
            g.graph.replay()
        t2 = time.perf_counter()
        legacy.wait_stream(cs)
        t3 = time.perf_counter()
        host.append(((t1 - t0) * 1e6, (t2 - t1) * 1e6, (t3 - t2) * 1e6))
    torch.cuda.synchronize()
    print("host us per call (cs waits legacy, replay, legacy waits cs): "
          + "; ".join(f"{a_:.0f}/{b_:.0f}/{c_:.0f}" for a_, b_, c_ in host), flush=True)

    def nw_replay():
        with lrn._on_stream(wait_caller=False):
            lrn._run("train", loader, True, None)

    def nw_reset_replay():
        with lrn._on_stream(wait_caller=False):
            lrn.engine.reset_optimizer()
            lrn._run("train", loader, True, None)

    def nw_perm():
        with lrn._on_stream(wait_caller=False):
            lrn.engine.reset_optimizer()
            lrn._run("train", loader, True, loader.permutation(host=True))

    def nw_perm_readback():
        with lrn._on_stream(wait_caller=False):
            lrn.engine.reset_optimizer()
            lrn._readback(lrn._run("train", loader, True, loader.permutation(host=True)))

    def nw_all():
        with lrn._on_stream(wait_caller=False):
            lrn.engine.reset_optimizer()
            lrn._readback(lrn._run("train", loader, True, loader.permutation(host=True)))
            lrn._validate_async()

    # timed on the learner stream itself
    def timed_on(stream, fn, label):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(20):
            fn()
        e1.record(stream)
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / 20
        print(f"[on learner stream] {label}: {us:.0f} us = {us / steps:.1f} us/step", flush=True)

    def cs_replay():
        with torch.cuda.stream(cs):
            g.graph.replay()

    def cs_replay_event():
        with torch.cuda.stream(cs):
            g.graph.replay()
        cs.record_event()

    def cs_replay_legacy_waits():
        with torch.cuda.stream(cs):
            g.graph.replay()
        legacy.wait_stream(cs)

    def cs_replay_side_waits():
        with torch.cuda.stream(cs):
            g.graph.replay()
        side.wait_stream(cs)


    def cs_replay_private_waits():
        with torch.cuda.stream(cs):
            g.graph.replay()
        priv.wait_stream(cs)

    from p2pfl_amd.utils.streams import private_stream

    priv = private_stream(dev)
    hi = private_stream(dev, -1)

    def hi_replay_legacy_waits():
        with torch.cuda.stream(hi):
            g.graph.replay()
        legacy.wait_stream(hi)

    def hi_replay_private_waits():
        with torch.cuda.stream(hi):
            g.graph.replay()
        priv.wait_stream(hi)

    timed_on(hi, hi_replay_legacy_waits, "HIGH-priority stream: replay + legacy stream waits for it")
    timed_on(hi, hi_replay_private_waits, "HIGH-priority stream: replay + private stream waits for it")
    timed_on(cs, cs_replay_side_waits, "replay + pooled stream waits for it")
    timed_on(cs, cs_replay_private_waits, "replay + private stream waits for it")
    timed_on(cs, cs_replay, "replay only")
    timed_on(cs, cs_replay_event, "replay + event record")
    timed_on(cs, cs_replay_legacy_waits, "replay + legacy stream waits for it")
    timed_on(cs, nw_replay, "_run under _on_stream(wait_caller=False)")

    for name, fn in (("no caller wait: replay", nw_replay),
                     ("no caller wait: + reset", nw_reset_replay),
                     ("no caller wait: + pinned batch order copy", nw_perm),
                     ("no caller wait: + stats readback", nw_perm_readback),
                     ("no caller wait: + validation", nw_all),
                     ("replay on the learner stream, no hand-off", on_cs_no_handoff),
                     ("replay on the learner stream, hand-off with the legacy default stream", on_cs_handoff_legacy),
                     ("replay on the learner stream, hand-off with a pooled stream", on_cs_handoff_side),
                     ("replay on the legacy default stream", on_legacy),
                     ("replay via _run on the learner stream", replay_on_stream),
                     ("+ optimizer reset", reset_replay),
                     ("+ pinned host batch order", reset_perm_replay),
                     ("+ device batch order (old path)", reset_devperm_replay),
                     ("epoch path (reset + copy + replay + readback)", epoch_only),
                     ("epoch path + validation", epoch_and_validation)):
        fn()
        torch.cuda.synchronize()
        a.record()
        for _ in range(20):
            fn()
        b.record()
        torch.cuda.synchronize()
        us = a.elapsed_time(b) * 1e3 / 20
        print(f"{name} x 20: {us:.0f} us each = {us / steps:.1f} us/step", flush=True)
    lrn.drain()
    # (2) fit() as the node calls it (reset, epoch, snapshots + validation on the side stream)
    a.record()
    for _ in range(20):
        lrn.fit()
    b.record()
    torch.cuda.synchronize()
    us = a.elapsed_time(b) * 1e3 / 20
    print(f"fit() x 20: {us:.0f} us per fit = {us / steps:.1f} us/step", flush=True)
    lrn.drain()


if __name__ == "__main__":
    main()
