"""Which part of a PyTorch-ROCm training step survives HIP graph capture?

    python tools/lab/graph_probe.py            # parent: runs every stage in a child, stops at the first crash
    python tools/lab/graph_probe.py <stage>    # one stage

Stages grow from a plain GEMM to the whole ResNet-18 step; each child warms
up on a side stream, captures, replays and checks against an eager run.
"""

from __future__ import annotations

import os
import subprocess
import sys

STAGES = ["linear", "conv_fwd", "conv_fwdbwd", "bn_fused", "resnet_fwd", "resnet_step_tl", "resnet_step_global",
          "resnet_step_tunable", "learner_notunable", "learner"]
if os.environ.get("PROBE_STAGES"):
    STAGES = os.environ["PROBE_STAGES"].split(",")


def stage(name: str) -> None:
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
    import torch
    from torch import nn

    torch.backends.cudnn.benchmark = True
    dev = torch.device("cuda", 0)
    cl = torch.channels_last
    torch.manual_seed(0)
    mode = "global" if name.endswith("_global") else "thread_local"

    if name.startswith("learner"):
        if name == "learner_notunable":
            os.environ["P2PFL_TUNABLEOP"] = "0"
        from p2pfl_amd.data import Cifar10FederatedDM
        from p2pfl_amd.learning.torch_learner import TorchLearner
        from p2pfl_amd.models.resnet import ResNet18

        ln = TorchLearner(ResNet18(seed=0), Cifar10FederatedDM(sub_id=0, number_sub=200, batch_size=32), "p", 1, device=dev)
        print(f"[{name}] mixed={ln.mixed}", flush=True)
        ln.fit()
        torch.cuda.synchronize()
        print(f"[{name}] fit ok, graph={ln._step_graph is not None}", flush=True)
        ln.fit()
        torch.cuda.synchronize()
        print(f"[{name}] second fit ok", flush=True)
        return
    if name == "resnet_step_tunable":
        from p2pfl_amd.tuning import enable_tuned_gemms

        print(f"[{name}] tunable={enable_tuned_gemms()}", flush=True)
    if name == "linear":
        m = nn.Linear(512, 256).to(dev)
        x = torch.randn(32, 512, device=dev)
        fn = lambda: m(x).sum()  # noqa: E731
        train = False
    elif name in ("conv_fwd", "conv_fwdbwd"):
        m = nn.Conv2d(64, 64, 3, 1, 1, bias=False).to(dev).to(memory_format=cl)
        x = torch.randn(32, 64, 32, 32, device=dev).to(memory_format=cl).requires_grad_(name == "conv_fwdbwd")

        def fn():
            with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
                y = m(x).float().sum()
            if name == "conv_fwdbwd":
                y.backward()
            return y

        train = name == "conv_fwdbwd"
    elif name == "bn_fused":
        from p2pfl_amd.ops.batchnorm import batch_norm_act

        bn = nn.BatchNorm2d(64).to(dev)
        x = torch.randn(32, 64, 16, 16, device=dev).to(torch.bfloat16).to(memory_format=cl).requires_grad_(True)

        def fn():
            y = batch_norm_act(x, bn).float().sum()
            y.backward()
            return y

        train = True
    else:
        from p2pfl_amd.models.resnet import ResNet18

        m = ResNet18(seed=0).to(dev)
        x = torch.randint(0, 255, (32, 3, 32, 32), dtype=torch.uint8, device=dev)
        t = torch.randint(0, 10, (32,), device=dev)
        train = name != "resnet_fwd"
        if not train:
            m.eval()

        def fn():
            with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
                loss = nn.functional.cross_entropy(m(x), t)
            if train:
                for p in m.parameters():
                    p.grad = None
                loss.backward()
            return loss.detach()

    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            ref = fn()
    torch.cuda.synchronize()
    print(f"[{name}] warmup ok", flush=True)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s, capture_error_mode=mode):
        out = fn()
    print(f"[{name}] capture ok", flush=True)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    print(f"[{name}] replay ok: {float(out):.5f} (eager {float(ref):.5f}) train={train}", flush=True)


def main() -> int:
    if len(sys.argv) > 1:
        stage(sys.argv[1])
        return 0
    env = dict(os.environ, AMD_LOG_LEVEL=os.environ.get("AMD_LOG_LEVEL", "1"))
    for name in STAGES:
        r = subprocess.run([sys.executable, __file__, name], env=env, timeout=300)
        print(f"== stage {name}: exit {r.returncode}", flush=True)
        if r.returncode != 0:
            return 1  # a crash ends the probe: nothing more runs on the GPU
    return 0


if __name__ == "__main__":
    sys.exit(main())
