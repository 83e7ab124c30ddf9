"""Count the layout/dtype fix-ups the fused BatchNorm backward inserts in a ResNet step (GPU)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from p2pfl_amd.models.resnet import ResNet18  # noqa: E402
from p2pfl_amd.ops import batchnorm as bnm  # noqa: E402

torch.backends.cudnn.benchmark = True
m = ResNet18(seed=0).cuda()
x = torch.randint(0, 255, (32, 3, 32, 32), dtype=torch.uint8, device="cuda")
y = torch.randint(0, 10, (32,), device="cuda")
for it in range(3):
    with torch.autocast("cuda", dtype=torch.bfloat16):
        loss = torch.nn.functional.cross_entropy(m(x), y)
    loss.backward()
    torch.cuda.synchronize()
    print(it, dict(bnm.STATS), flush=True)
# which layers produce non-channels-last gradients?
seen = []
for name, mod in m.named_modules():
    if isinstance(mod, torch.nn.Conv2d):
        mod.register_full_backward_hook(lambda mo, gi, go, n=name: seen.append((n, [g.is_contiguous(memory_format=torch.channels_last) if g is not None else None for g in gi], [g.is_contiguous(memory_format=torch.channels_last) for g in go if g is not None])))
with torch.autocast("cuda", dtype=torch.bfloat16):
    loss = torch.nn.functional.cross_entropy(m(x), y)
loss.backward()
for s in seen[:12]:
    print(s)
