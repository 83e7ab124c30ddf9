"""Numerics of the HIP kernels vs plain-PyTorch fp32 references (MI355X only)."""

from __future__ import annotations

import pytest
import torch

from p2pfl_amd import ops
from p2pfl_amd.learning.optim import mt_layout

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _require_ext():
    ops.ext()  # fail loudly if the native extension is missing on a GPU box


@pytest.mark.parametrize("k", [1, 2, 3, 8, 16, 21])
@pytest.mark.parametrize("n", [64, 4096 + 4, 6_497_216])
def test_weighted_sum(k, n):
    g = torch.Generator(device="cuda").manual_seed(k * 7 + n % 13)
    flats = [torch.randn(n, device="cuda", generator=g) for _ in range(k)]
    weights = [float(i % 5 + 1) for i in range(k)]
    out = ops.weighted_average(flats, weights)
    ref = ops.weighted_average_reference([f.double() for f in flats], weights).float()
    torch.testing.assert_close(out, ref, atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("in_dtypes", ["f32", "bf16", "mixed"])
@pytest.mark.parametrize("out_dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("k,n", [(1, 4096 + 3), (3, 6_497_216), (8, 1 << 20), (21, 777)])
def test_weighted_sum_dtypes(in_dtypes, out_dtype, k, n):
    """bf16 arenas (bf16 wire option) are averaged directly: fp32 accumulation,
    fp32 or bf16 result, against an fp64 reference of the same (bf16-valued) inputs."""
    g = torch.Generator(device="cuda").manual_seed(k + n % 11)
    flats = []
    for i in range(k):
        f = torch.randn(n, device="cuda", generator=g)
        if in_dtypes == "bf16" or (in_dtypes == "mixed" and i % 2):
            f = f.to(torch.bfloat16)
        flats.append(f)
    weights = [float(i % 4 + 1) for i in range(k)]
    out = ops.weighted_average(flats, weights, out_dtype=out_dtype)
    assert out.dtype == out_dtype
    ref = ops.weighted_average_reference([f.double() for f in flats], weights)
    if out_dtype == torch.bfloat16:
        torch.testing.assert_close(out, ref.to(torch.bfloat16), atol=1e-2, rtol=8e-3)
    else:
        torch.testing.assert_close(out, ref.float(), atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("decoupled,wd", [(False, 0.0), (False, 0.01), (True, 0.1)])
def test_adam_step(decoupled, wd):
    n = 1 << 20
    torch.manual_seed(0)
    p = torch.randn(n, device="cuda")
    m = torch.zeros(n, device="cuda")
    v = torch.zeros(n, device="cuda")
    p_ref, m_ref, v_ref = p.clone(), m.clone(), v.clone()
    shadow = torch.empty(n, device="cuda", dtype=torch.bfloat16)
    for step in range(1, 4):
        g = torch.randn(n, device="cuda")
        ops.adam_step(p, g, m, v, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=wd, step=step, decoupled=decoupled, p_bf16=shadow)
        ops.adam_step_reference(p_ref, g, m_ref, v_ref, 1e-3, 0.9, 0.999, 1e-8, wd, step, decoupled)
    torch.testing.assert_close(p, p_ref, atol=1e-6, rtol=1e-5)
    torch.testing.assert_close(m, m_ref, atol=1e-6, rtol=1e-5)
    torch.testing.assert_close(v, v_ref, atol=1e-7, rtol=1e-5)
    torch.testing.assert_close(shadow, p.to(torch.bfloat16), atol=0, rtol=0)


@pytest.mark.parametrize("momentum,nesterov", [(0.0, False), (0.9, False), (0.9, True)])
def test_sgd_step(momentum, nesterov):
    n = 1 << 18
    torch.manual_seed(1)
    p = torch.randn(n, device="cuda")
    buf = torch.zeros(n, device="cuda") if momentum else None
    p_ref = p.clone()
    buf_ref = buf.clone() if buf is not None else None
    for step in range(3):
        g = torch.randn(n, device="cuda")
        ops.sgd_step(p, g, buf, lr=0.1, momentum=momentum, weight_decay=1e-4, nesterov=nesterov, first_step=step == 0)
        ops.sgd_step_reference(p_ref, g, buf_ref, 0.1, momentum, 0.0, 1e-4, nesterov, step == 0)
    torch.testing.assert_close(p, p_ref, atol=1e-6, rtol=1e-5)


def test_fedavg_uses_kernel_on_gpu():
    from collections import OrderedDict

    from p2pfl_amd.learning.aggregators import FedAvg
    from p2pfl_amd.learning.arena import flatten

    a = flatten(OrderedDict(w=torch.ones(100, device="cuda"), b=torch.zeros(3, device="cuda")))
    b = flatten(OrderedDict(w=torch.full((100,), 3.0, device="cuda"), b=torch.ones(3, device="cuda")))
    res = FedAvg().aggregate({"a": (a, 1), "b": (b, 3)})
    assert res.flat.is_cuda
    torch.testing.assert_close(res["w"], torch.full((100,), 2.5, device="cuda"))
    torch.testing.assert_close(res["b"], torch.full((3,), 0.75, device="cuda"))


class _Tables:
    """Minimal MTTables stand-in: tensors at 64-aligned offsets of one arena."""

    def __init__(self, sizes, bf16_flags, dev, cl=None):
        self.table, off = [], 0
        cl = cl or [None] * len(sizes)
        for t, (n, bf) in enumerate(zip(sizes, bf16_flags)):
            flags = (1 if bf else 0) | (2 if bf else 0)
            if cl[t] is not None:  # (in_channels, kh*kw): channels-last grad + shadow
                flags |= 4 | (cl[t][0] << 8) | (cl[t][1] << 32)
            self.table.append((off, n, flags))
            off = (off + n + 63) // 64 * 64
        self.numel = max(off, 64)
        self.numels = list(sizes)
        self.grad_bf16 = list(bf16_flags)
        self.grad_cl = [c is not None for c in cl]
        self.tens, self.chunks = mt_layout(self.table, dev)


@pytest.mark.parametrize("decoupled,wd", [(False, 0.01), (True, 0.05)])
def test_adam_multi_tensor(decoupled, wd):
    sizes = [3, 4096, 4099, 768 * 3072 + 5, 1, 10_000]
    bf = [False, True, True, True, False, False]
    mt = _Tables(sizes, bf, "cuda")
    torch.manual_seed(2)
    p = torch.randn(mt.numel, device="cuda")
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    shadow = torch.zeros(mt.numel, device="cuda", dtype=torch.bfloat16)
    p_ref, m_ref, v_ref, s_ref = p.clone(), m.clone(), v.clone(), shadow.clone()
    for step in range(1, 4):
        grads = [torch.randn(n, device="cuda", dtype=torch.bfloat16 if b else torch.float32) for n, b in zip(sizes, bf)]
        if step == 2:
            grads[1] = None  # skipped this step
        kw = dict(lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=wd, step=step, decoupled=decoupled)
        ops.adam_mt_step(p, m, v, grads, mt, p_bf16=shadow, **kw)
        ops._mt_reference(
            lambda pp, g, mm, vv: ops.adam_step_reference(pp, g, mm, vv, 1e-3, 0.9, 0.999, 1e-8, wd, step, decoupled),
            p_ref, (m_ref, v_ref), s_ref, mt.table, grads,
        )
    torch.testing.assert_close(p, p_ref, atol=1e-6, rtol=1e-5)
    torch.testing.assert_close(m, m_ref, atol=1e-6, rtol=1e-5)
    torch.testing.assert_close(v, v_ref, atol=1e-7, rtol=5e-5)  # fma contraction
    for off, n, flags in mt.table:  # the shadow is the kernel's own fp32 result rounded to bf16
        want = p[off:off + n].to(torch.bfloat16) if flags & 2 else torch.zeros(n, device="cuda", dtype=torch.bfloat16)
        assert torch.equal(shadow[off:off + n], want)


def test_sgd_multi_tensor():
    sizes = [5, 4096 * 3 + 17, 64]
    bf = [False, True, False]
    mt = _Tables(sizes, bf, "cuda")
    torch.manual_seed(3)
    p = torch.randn(mt.numel, device="cuda")
    buf = torch.zeros_like(p)
    shadow = torch.zeros(mt.numel, device="cuda", dtype=torch.bfloat16)
    p_ref, b_ref, s_ref = p.clone(), buf.clone(), shadow.clone()
    for step in range(3):
        grads = [torch.randn(n, device="cuda", dtype=torch.bfloat16 if b else torch.float32) for n, b in zip(sizes, bf)]
        kw = dict(lr=0.1, momentum=0.9, dampening=0.0, weight_decay=1e-4, nesterov=True, first_step=step == 0)
        ops.sgd_mt_step(p, buf, grads, mt, p_bf16=shadow, **kw)
        ops._mt_reference(
            lambda pp, g, b: ops.sgd_step_reference(pp, g, b, 0.1, 0.9, 0.0, 1e-4, True, step == 0),
            p_ref, (b_ref,), s_ref, mt.table, grads,
        )
    torch.testing.assert_close(p, p_ref, atol=1e-6, rtol=1e-5)
    torch.testing.assert_close(shadow, s_ref, atol=0, rtol=0)


def test_multi_tensor_rejects_bad_grads():
    mt = _Tables([100], [False], "cuda")
    p = torch.zeros(mt.numel, device="cuda")
    with pytest.raises(RuntimeError):
        ops.adam_mt_step(p, p.clone(), p.clone(), [torch.zeros(99, device="cuda")], mt, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.0, step=1)
    with pytest.raises(RuntimeError):
        ops.adam_mt_step(p, p.clone(), p.clone(), [torch.zeros(100, device="cuda", dtype=torch.bfloat16)], mt, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.0, step=1)


@pytest.mark.parametrize("model", ["mlp", "vit_tiny", "resnet18"])
def test_gpu_learner_uses_mixed_precision(model):
    """The GPU TorchLearner runs bf16 weight shadows + one multi-tensor optimizer launch, and learns."""
    from p2pfl_amd.data import Cifar10FederatedDM, MnistFederatedDM
    from p2pfl_amd.learning.torch_learner import TorchLearner
    from p2pfl_amd.models import MLP
    from p2pfl_amd.models.resnet import ResNet18
    from p2pfl_amd.models.vit import ViT_Tiny

    if model == "mlp":
        m, dm = MLP(seed=0), MnistFederatedDM(sub_id=0, number_sub=20)
    elif model == "vit_tiny":
        m, dm = ViT_Tiny(seed=0), Cifar10FederatedDM(sub_id=0, number_sub=40)
    else:
        m, dm = ResNet18(num_classes=10, seed=0), Cifar10FederatedDM(sub_id=0, number_sub=40)
    nl = TorchLearner(m, dm, "gpu-mixed", 1, device="cuda")
    assert nl.mixed and nl.arena.shadow is not None and nl.arena.shadow_names
    ev0 = nl.evaluate()["test_loss"]
    nl.fit()
    torch.cuda.synchronize()
    params = nl.get_parameters()
    assert all(torch.isfinite(v).all() for v in params.values())
    for name in nl.arena.shadow_names:
        w = dict(nl.model.named_parameters())[name]
        assert w.dtype == torch.bfloat16
        assert torch.equal(w.detach(), params[name].to(torch.bfloat16)), name
    if model != "resnet18":  # ResNet eval on a Dirichlet shard after 1 epoch is noisy
        assert nl.evaluate()["test_loss"] < ev0


@pytest.mark.parametrize("opt", ["adam", "sgd"])
def test_multi_tensor_channels_last(opt):
    """Conv weights with channels-last grads/shadows: fp32 state in OIHW order, shadow written at OHWI positions."""
    # staged through LDS (csrc/optim.hip ClStage): 64x32x3x3 (slab 288: 16 slabs per chunk), 128x64x5x5
    # (slab 1600: 2 per chunk), 512x512x3x3 (one 4608 slab per chunk), 40x36x3x3 (slab 324: 14 per
    # chunk); gather path: 16x3x7x7 (I = 3), 8x1024x3x3 and 8x192x5x5 (slabs 9216 / 4800 > 4608:
    # plain chunks that start mid-slab); no permutation: 24x8x1x1
    shapes = [(64, 32, 3, 3), (10, 7), (128, 64, 5, 5), (16, 3, 7, 7), (512, 512, 3, 3), (40, 36, 3, 3), (24, 8, 1, 1),
              (8, 1024, 3, 3), (8, 192, 5, 5)]
    cl = [(s[1], s[2] * s[3]) if len(s) == 4 else None for s in shapes]
    sizes = [int(torch.Size(s).numel()) for s in shapes]
    mt = _Tables(sizes, [True] * len(shapes), "cuda", cl=cl)
    torch.manual_seed(5)
    p = torch.randn(mt.numel, device="cuda")
    st = [torch.zeros_like(p), torch.zeros_like(p)]
    shadow = torch.zeros(mt.numel, device="cuda", dtype=torch.bfloat16)
    p_ref, st_ref, s_ref = p.clone(), [t.clone() for t in st], shadow.clone()
    for step in range(1, 4):
        grads = []
        for s in shapes:
            g = torch.randn(s, device="cuda").to(torch.bfloat16)
            grads.append(g.contiguous(memory_format=torch.channels_last) if len(s) == 4 else g)
        if opt == "adam":
            kw = dict(lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.01, step=step)
            ops.adam_mt_step(p, st[0], st[1], grads, mt, p_bf16=shadow, **kw)
            ops._mt_reference(
                lambda pp, g, mm, vv: ops.adam_step_reference(pp, g, mm, vv, 1e-3, 0.9, 0.999, 1e-8, 0.01, step, False),
                p_ref, tuple(st_ref), s_ref, mt.table, grads,
            )
        else:
            kw = dict(lr=0.05, momentum=0.9, dampening=0.0, weight_decay=5e-4, nesterov=False, first_step=step == 1)
            ops.sgd_mt_step(p, st[0], grads, mt, p_bf16=shadow, **kw)
            ops._mt_reference(
                lambda pp, g, b: ops.sgd_step_reference(pp, g, b, 0.05, 0.9, 0.0, 5e-4, False, step == 1),
                p_ref, (st_ref[0],), s_ref, mt.table, grads,
            )
    torch.testing.assert_close(p, p_ref, atol=1e-6, rtol=1e-5)
    for (off, n, _), s in zip(mt.table, shapes):
        want = p[off:off + n].view(s).to(torch.bfloat16)
        got = shadow[off:off + n]
        if len(s) == 4:  # channels-last region: memory order (O, kh, kw, I)
            got = got.view(s[0], s[2], s[3], s[1]).permute(0, 3, 1, 2)
        assert torch.equal(got.reshape(s), want)
    with pytest.raises(RuntimeError):  # an OIHW-contiguous gradient is rejected for a channels-last tensor
        bad = [g.contiguous() for g in grads]
        ops.sgd_mt_step(p, st[0], bad, mt, lr=0.05, momentum=0.9, p_bf16=shadow)


@pytest.mark.gpu
def test_weighted_sum_running_fold_is_bitwise_equal_to_one_shot():
    """The FedAvg kernel seeded with a running fp32 sum (acc_in) and scaled at
    the end: folding inputs in pieces equals one launch bit for bit, including
    bf16 inputs, a zero-input scale-only launch and > 16 inputs."""
    from p2pfl_amd import ops

    ops.ext()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(5)
    n = 6_497_163  # not a multiple of 4: the tail kernel runs too
    flats = [torch.randn(n, device=dev, generator=g) for _ in range(19)]
    flats[3] = flats[3].to(torch.bfloat16)
    w = [float(100 + 13 * i) for i in range(19)]
    scale = 1.0 / sum(w)
    one = torch.empty(n, device=dev)
    ops.weighted_sum_into(one, flats, w, None, scale)
    acc = torch.empty(n, device=dev)
    ops.weighted_sum_into(acc, flats[:2], w[:2])
    ops.weighted_sum_into(acc, flats[2:7], w[2:7], acc_in=acc)
    ops.weighted_sum_into(acc, flats[7:], w[7:], acc_in=acc)
    out = torch.empty(n, device=dev)
    ops.weighted_sum_into(out, [], [], acc_in=acc, scale=scale)
    assert torch.equal(out, one)
    ref = sum(f.double() * wi for f, wi in zip(flats, w)) * scale
    torch.testing.assert_close(one.double(), ref, rtol=1e-5, atol=1e-5)
    # the wrapper FedAvg uses
    torch.testing.assert_close(ops.weighted_average(flats, w), one, rtol=0, atol=0)


def test_multi_copy_regions():
    """fused.multi_copy: every (dst, src) pair copied in one launch, dword tails included, dtypes mixed."""
    C = ops.ext().fused
    g = torch.Generator(device="cuda").manual_seed(0)
    srcs = [torch.randn(n, device="cuda", generator=g) for n in (3, 4, 17, 4096 + 5, 1 << 20)]
    srcs.append(torch.randn(6002, device="cuda", generator=g).to(torch.bfloat16))
    dsts = [torch.zeros_like(s) for s in srcs]
    C.multi_copy(dsts, srcs)
    for d, s in zip(dsts, srcs):
        assert torch.equal(d, s)
    with pytest.raises(RuntimeError):
        C.multi_copy([torch.zeros(4, device="cuda")], [torch.zeros(5, device="cuda")])
