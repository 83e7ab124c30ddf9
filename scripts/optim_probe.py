"""Time the multi-tensor SGD / Adam launches on ResNet-18's parameter set.

Conv weights are channels-last (bf16 gradient and shadow in (O, kh, kw, I) order,
fp32 master and state in OIHW order), everything else plain -- the layout the
mixed-precision learner hands `ops.sgd_mt_step` / `ops.adam_mt_step`.

    python scripts/optim_probe.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from p2pfl_amd import ops  # noqa: E402
from p2pfl_amd.learning.optim import mt_layout  # noqa: E402
from p2pfl_amd.models.resnet import ResNet18, ResNet50  # noqa: E402


class Tables:
    def __init__(self, shapes, dev):
        self.table, off = [], 0
        self.numels, self.grad_bf16, self.grad_cl = [], [], []
        for s in shapes:
            n = int(torch.Size(s).numel())
            flags = 1 | 2
            cl = len(s) == 4 and s[2] * s[3] > 1
            if cl:
                flags |= 4 | (s[1] << 8) | ((s[2] * s[3]) << 32)
            self.table.append((off, n, flags))
            off = (off + n + 63) // 64 * 64
            self.numels.append(n)
            self.grad_bf16.append(True)
            self.grad_cl.append(cl)
        self.numel = off
        self.tens, self.chunks = mt_layout(self.table, dev)


def timeit(fn, iters=50, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / iters


def main():
    dev = torch.device("cuda")
    for name, net in (("resnet18", ResNet18), ("resnet50", ResNet50)):
        shapes = [tuple(p.shape) for p in net(seed=0).parameters()]
        mt = Tables(shapes, dev)
        p = torch.randn(mt.numel, device=dev)
        buf, m, v = torch.zeros_like(p), torch.zeros_like(p), torch.zeros_like(p)
        shadow = torch.zeros(mt.numel, device=dev, dtype=torch.bfloat16)
        grads = []
        for s in shapes:
            g = torch.randn(s, device=dev).to(torch.bfloat16)
            grads.append(g.contiguous(memory_format=torch.channels_last) if len(s) == 4 and s[2] * s[3] > 1 else g)
        # persistent gradient-address table (as the captured training step uses): no per-call upload
        gtab = torch.tensor([g.data_ptr() for g in grads], dtype=torch.int64, device=dev)
        sgd = timeit(lambda: ops.sgd_mt_step(p, buf, grads, mt, lr=0.05, momentum=0.9, weight_decay=5e-4, p_bf16=shadow,
                                             gtab=gtab))
        adam = timeit(lambda: ops.adam_mt_step(p, m, v, grads, mt, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8,
                                               weight_decay=0.0, step=1, p_bf16=shadow, gtab=gtab))
        n = sum(mt.numels)
        # bytes: SGD reads p, buf (fp32) + grad (bf16), writes p, buf + shadow (bf16) = 20 B / param;
        # Adam reads p, m, v + grad, writes p, m, v + shadow = 28 B / param
        print(json.dumps({"model": name, "params": n, "sgd_mt_us": round(sgd, 2), "sgd_TBps": round(20 * n / sgd / 1e6, 2),
                          "adam_mt_us": round(adam, 2), "adam_TBps": round(28 * n / adam / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
