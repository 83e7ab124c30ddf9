"""Learner / aggregator / codec tests (reference ``test/learning_test.py`` + property tests)."""

from __future__ import annotations

import itertools
import pickle
import random
from collections import OrderedDict

import pytest
import torch

from p2pfl_amd.learning.aggregators import FedAvg
from p2pfl_amd.learning.arena import FlatParams, ModuleArena, ParamLayout, flatten
from p2pfl_amd.learning.exceptions import DecodingParamsError, ModelNotMatchingError
from p2pfl_amd.learning.torch_learner import LightningLearner, TorchLearner
from p2pfl_amd.learning.wire import decode_params, encode_params
from p2pfl_amd.models import CNN, MLP


def test_encoding():
    nl1 = TorchLearner(MLP(), None, "", 1, device="cpu")
    encoded = nl1.encode_parameters()
    nl2 = LightningLearner(MLP(), None, "", 1, device="cpu")
    nl2.set_parameters(nl2.decode_parameters(encoded))
    assert encoded == nl2.encode_parameters()


def test_avg_simple():
    agg = FedAvg()
    a = OrderedDict([("a", torch.tensor(-1)), ("b", torch.tensor(-1))])
    b = OrderedDict([("a", torch.tensor(0)), ("b", torch.tensor(0))])
    c = OrderedDict([("a", torch.tensor(1)), ("b", torch.tensor(1))])
    res = agg.aggregate({"a": (a, 1), "b": (b, 1), "c": (c, 1)})
    for layer in b:
        assert res[layer] == b[layer]
    res = agg.aggregate({"a": (a, 1), "b": (b, 7), "c": (c, 1)})
    for layer in b:
        assert res[layer] == b[layer]
    res = agg.aggregate({"a": (a, 800), "b": (b, 0), "c": (c, 0)})
    for layer in b:
        assert res[layer] == a[layer]


def test_avg_complex():
    agg = FedAvg()
    nl = TorchLearner(MLP(), None, "", 1, device="cpu")
    params = {k: v.clone() for k, v in nl.get_parameters().items()}
    res = agg.aggregate({"a": (params, 1)})
    for layer in params:
        assert torch.eq(params[layer], res[layer]).all()
    p1 = {k: v + 1 for k, v in params.items()}
    p2 = {k: v - 1 for k, v in params.items()}
    res = agg.aggregate({"a": (p1, 1), "b": (p2, 1)})
    for layer in params:
        assert torch.allclose(params[layer], res[layer], atol=1e-5)


@pytest.mark.parametrize("seed", range(5))
def test_partial_aggregation_equals_fedavg(seed):
    """Any disjoint partition, partially aggregated then combined, equals one-shot FedAvg."""
    rng = random.Random(seed)
    nodes = [f"n{i}" for i in range(6)]
    models = {n: OrderedDict(w=torch.randn(33), b=torch.randn(4, 5)) for n in nodes}
    weights = {n: rng.randint(1, 100) for n in nodes}
    full = FedAvg().aggregate({n: (models[n], weights[n]) for n in nodes})
    # random disjoint partition into partial aggregates
    order = nodes[:]
    rng.shuffle(order)
    cuts = sorted(rng.sample(range(1, 6), 2))
    groups = [order[: cuts[0]], order[cuts[0] : cuts[1]], order[cuts[1] :]]
    agg = FedAvg("me")
    agg.set_nodes_to_aggregate(nodes)
    for g in groups:
        sub = FedAvg().aggregate({n: (models[n], weights[n]) for n in g})
        assert agg.add_model(sub, g, sum(weights[n] for n in g))
    combined = agg.wait_and_get_aggregation(timeout=1)
    for k in full:
        assert torch.allclose(full[k], combined[k], atol=1e-5)


def test_aggregator_rules():
    agg = FedAvg("me")
    m = OrderedDict(w=torch.ones(3))
    agg.set_nodes_to_aggregate(["a", "b", "c"])
    with pytest.raises(Exception):
        agg.set_nodes_to_aggregate(["a"])
    assert agg.add_model(m, [], 1) == []  # Q4: empty contributors
    assert agg.add_model(m, ["x"], 1) == []  # not in train set
    assert agg.add_model(m, ["a"], 1) == ["a"]
    assert agg.would_accept(["b"]) and not agg.would_accept(["a", "b"])
    assert agg.add_model(m, ["a", "b"], 1) == []  # overlap
    assert sorted(agg.add_model(m, ["b", "c"], 2)) == ["a", "b", "c"]
    assert agg.add_model(m, ["c"], 1) == []  # not needed anymore
    agg.clear()
    # a full model replaces partial ones
    agg.set_nodes_to_aggregate(["a", "b"])
    agg.add_model(OrderedDict(w=torch.zeros(3)), ["a"], 1)
    agg.add_model(OrderedDict(w=torch.full((3,), 5.0)), ["a", "b"], 2)
    res = agg.wait_and_get_aggregation(timeout=1)
    assert torch.allclose(res["w"], torch.full((3,), 5.0))
    agg.clear()


def test_waiting_aggregated_model_timeout_returns_none():
    agg = FedAvg("me")
    agg.set_waiting_aggregated_model(["a", "b"])
    assert agg.add_model(OrderedDict(w=torch.ones(2)), ["a"], 1) == []  # only the full aggregate is accepted
    assert agg.wait_and_get_aggregation(timeout=0.2) is None  # Q5: keep local model
    agg.clear()
    agg.set_waiting_aggregated_model(["a", "b"])
    assert agg.add_model(OrderedDict(w=torch.ones(2)), ["b", "a"], 1) == ["b", "a"]
    assert torch.equal(agg.wait_and_get_aggregation(timeout=1)["w"], torch.ones(2))


def test_partial_aggregation_excludes_and_caches():
    agg = FedAvg("me")
    agg.set_nodes_to_aggregate(["a", "b", "c"])
    agg.add_model(OrderedDict(w=torch.full((4,), 1.0)), ["a"], 1)
    agg.add_model(OrderedDict(w=torch.full((4,), 3.0)), ["b"], 3)
    m, contrib, w = agg.get_partial_aggregation(["c"])
    assert sorted(contrib) == ["a", "b"] and w == 4 and torch.allclose(m["w"], torch.full((4,), 2.5))
    m2, _, _ = agg.get_partial_aggregation(["c"])
    assert m2 is m  # memoised
    m3, contrib3, w3 = agg.get_partial_aggregation(["a"])
    assert contrib3 == ["b"] and w3 == 3
    assert agg.get_partial_aggregation(["a", "b"]) == (None, None, None)


def test_wire_codec_roundtrip_and_safety():
    params = OrderedDict(
        a=torch.randn(3, 4), b=torch.arange(5, dtype=torch.int64), c=torch.randn(2).to(torch.bfloat16), d=torch.tensor(True)
    )
    out = decode_params(encode_params(params))
    for k in params:
        assert out[k].dtype == params[k].dtype and torch.equal(out[k], params[k])
    flat = flatten(OrderedDict(x=torch.randn(10), y=torch.randn(3, 3)))
    back = decode_params(encode_params(flat))
    assert isinstance(back, FlatParams) and torch.equal(back.flat, flat.flat) and back.layout == flat.layout
    # a pickle payload (what the reference sends) is read by the allow-listed
    # decoder (numeric arrays only); anything executable is refused, never run
    got = decode_params(pickle.dumps([torch.arange(3.0).numpy()]))
    assert isinstance(got, list) and torch.equal(got[0], torch.arange(3.0))
    with pytest.raises(DecodingParamsError):
        decode_params(pickle.dumps([print]))
    with pytest.raises(DecodingParamsError):
        decode_params(encode_params(flat)[:-8])


def test_decode_wrong_model_raises():
    mlp = TorchLearner(MLP(), None, "", 1, device="cpu")
    cnn = TorchLearner(CNN(), None, "", 1, device="cpu")
    with pytest.raises(ModelNotMatchingError):
        mlp.decode_parameters(cnn.encode_parameters())
    with pytest.raises(ModelNotMatchingError):
        mlp.set_parameters(cnn.get_parameters())


def test_arena_binding_is_live():
    model = MLP()
    arena = ModuleArena(model, grads=True)
    assert arena.layout.names == tuple(model.state_dict().keys())
    arena.flat.zero_()
    assert float(model.l1.weight.abs().sum()) == 0.0
    x = torch.randn(4, 1, 28, 28)
    model(x).sum().backward()
    assert arena.grads_bound() and float(arena.grads.abs().sum()) > 0


def test_layout_alignment():
    lay = ParamLayout.from_tensors([("a", torch.zeros(3)), ("b", torch.zeros(70)), ("c", torch.zeros(1))])
    assert lay.offsets == (0, 64, 192) and lay.numel == 256


@pytest.mark.parametrize("opt_name", ["adam", "adamw", "sgd", "sgd_nesterov"])
def test_fused_optimizer_matches_torch(opt_name):
    from p2pfl_amd.learning.optim import fuse_optimizer

    torch.manual_seed(0)
    m1, m2 = MLP(), MLP()
    m2.load_state_dict(m1.state_dict())
    mk = {
        "adam": lambda p: torch.optim.Adam(p, lr=1e-2, weight_decay=0.01),
        "adamw": lambda p: torch.optim.AdamW(p, lr=1e-2, weight_decay=0.1),
        "sgd": lambda p: torch.optim.SGD(p, lr=0.1, momentum=0.9, weight_decay=1e-3),
        "sgd_nesterov": lambda p: torch.optim.SGD(p, lr=0.1, momentum=0.9, nesterov=True),
    }[opt_name]
    ref_opt = mk(m1.parameters())
    arena = ModuleArena(m2, grads=True)
    fused = fuse_optimizer(mk(m2.parameters()), arena)
    assert fused is not None
    for step in range(3):
        x = torch.randn(8, 1, 28, 28)
        y = torch.randint(0, 10, (8,))
        for m, o in ((m1, ref_opt), (m2, fused)):
            o.zero_grad()
            torch.nn.functional.nll_loss(m(x), y).backward()
            o.step()
    for (k, a), b in zip(m1.state_dict().items(), m2.state_dict().values()):
        assert torch.allclose(a, b, atol=1e-5, rtol=1e-4), k


def test_learner_fit_evaluate_cpu():
    from p2pfl_amd.data import MnistFederatedDM
    from p2pfl_amd.management.logger import logger

    dm = MnistFederatedDM(sub_id=0, number_sub=40)
    nl = TorchLearner(MLP(seed=1), dm, "learner-test", 1, device="cpu")
    assert nl.get_num_samples() == (1350, 250)
    logger.register_node("learner-test", type("S", (), {"round": 0, "actual_exp_name": "exp"})(), True)
    try:
        before = nl.evaluate()
        nl.fit()
        after = nl.evaluate()
    finally:
        logger.unregister_node("learner-test")
    assert after["test_loss"] < before["test_loss"]
    assert after["test_metric"] > 0.3


def test_aggregator_lost_members():
    """A train-set member that leaves mid-round stops being waited for (trainer and waiting node)."""
    import torch

    from p2pfl_amd.learning.aggregators import FedAvg

    t = lambda v: {"w": torch.full((4,), float(v))}  # noqa: E731
    agg = FedAvg("a")
    agg.set_nodes_to_aggregate(["a", "b", "c"])
    agg.add_model(t(1), ["a"], 1)
    agg.add_model(t(3), ["b"], 1)
    assert not agg._done.is_set()
    agg.mark_lost(["c"])
    assert agg._done.is_set()
    out = agg.wait_and_get_aggregation(timeout=0.1)
    assert torch.allclose(out["w"], torch.full((4,), 2.0))
    # an aggregate of every live member supersedes overlapping partials
    agg.clear()
    agg.set_nodes_to_aggregate(["a", "b", "c", "d"])
    agg.mark_lost(["d"])
    agg.add_model(t(1), ["a"], 1)
    assert agg.would_accept(["a", "b", "c"])
    assert agg.add_model(t(5), ["a", "b", "c"], 3)
    assert agg._done.is_set()
    # a waiting (non-trainer) node accepts the aggregate of the live members
    w = FedAvg("w")
    w.set_waiting_aggregated_model(["a", "b", "c"])
    assert not w.would_accept(["a", "b"])
    w.mark_lost(["c"])
    assert w.would_accept(["a", "b"]) and w.add_model(t(7), ["a", "b"], 1)
    assert torch.equal(w.wait_and_get_aggregation(timeout=0.1)["w"], t(7)["w"])
    # a "lost" member whose model still arrives is accepted and un-marked
    x = FedAvg("x")
    x.set_nodes_to_aggregate(["a", "b", "c"])
    x.mark_lost(["c"])
    x.add_model(t(1), ["c"], 1)
    assert "c" in x.get_aggregated_models() and not x._lost


def test_aggregator_heartbeat_stall_member_comes_back():
    """A trainer evicted by a heartbeat stall (not a crash) that reappears before the
    aggregation completes is waited for again; once complete, the aggregate stays final."""
    t = lambda v: {"w": torch.full((4,), float(v))}  # noqa: E731
    agg = FedAvg("a")
    agg.set_nodes_to_aggregate(["a", "b", "c"])
    agg.add_model(t(1), ["a"], 1)
    agg.mark_lost(["c"])  # heartbeat timeout while c is still training
    agg.mark_alive(["c"])  # c's heartbeat is seen again
    agg.add_model(t(3), ["b"], 1)
    assert not agg._done.is_set()  # still waiting for c
    agg.add_model(t(5), ["c"], 1)
    assert torch.allclose(agg.wait_and_get_aggregation(timeout=0.1)["w"], torch.full((4,), 3.0))
    # completed without the member: a late reappearance does not reopen the round
    agg.clear()
    agg.set_nodes_to_aggregate(["a", "b", "c"])
    agg.add_model(t(1), ["a"], 1)
    agg.add_model(t(3), ["b"], 1)
    agg.mark_lost(["c"])
    assert agg._done.is_set()
    agg.mark_alive(["c"])
    assert agg._done.is_set() and "c" in agg._lost
    assert torch.allclose(agg.wait_and_get_aggregation(timeout=0.1)["w"], torch.full((4,), 2.0))


def test_mixed_precision_learner_cpu():
    """bf16 weight shadows + multi-tensor Adam (the GPU learner path) on the CPU reference ops."""
    from p2pfl_amd.data import MnistFederatedDM

    dm = MnistFederatedDM(sub_id=0, number_sub=40)
    nl = TorchLearner(MLP(seed=1), dm, "mixed-test", 1, device="cpu", precision="bf16", mixed=True)
    arena = nl.arena
    assert nl.mixed and arena.shadow is not None and arena.grads is None
    # matrix weights are bf16 views of the shadow; biases stay fp32 views of the master arena
    for name, p in nl.model.named_parameters():
        assert p.dtype == (torch.bfloat16 if p.dim() >= 2 else torch.float32), name
    before = {k: v.clone() for k, v in nl.get_parameters().items()}
    ev0 = nl.evaluate()["test_loss"]
    nl.fit()
    assert nl.evaluate()["test_loss"] < ev0
    params = nl.get_parameters()
    assert all(v.dtype == torch.float32 for v in params.values())
    assert any(not torch.equal(before[k], v) for k, v in params.items())
    for name in arena.shadow_names:  # shadow rewritten by every step
        w = dict(nl.model.named_parameters())[name]
        assert torch.equal(w.detach(), params[name].to(torch.bfloat16)), name
    # set_parameters refreshes the shadow
    nl.set_parameters(before)
    w = dict(nl.model.named_parameters())[arena.shadow_names[0]]
    assert torch.equal(w.detach(), before[arena.shadow_names[0]].to(torch.bfloat16))


@pytest.mark.parametrize("opt_name", ["adam", "adamw", "sgd"])
def test_multi_tensor_optimizer_matches_torch(opt_name):
    """MTAdam/MTSGD over per-tensor grads == torch.optim on the same fp32 grads."""
    from p2pfl_amd.learning.arena import ModuleArena
    from p2pfl_amd.learning.optim import fuse_optimizer_mt

    m1, m2 = MLP(seed=3), MLP(seed=3)
    make = {
        "adam": lambda ps: torch.optim.Adam(ps, lr=1e-2, weight_decay=1e-3),
        "adamw": lambda ps: torch.optim.AdamW(ps, lr=1e-2, weight_decay=0.05),
        "sgd": lambda ps: torch.optim.SGD(ps, lr=0.1, momentum=0.9, nesterov=True, weight_decay=1e-4),
    }[opt_name]
    arena = ModuleArena(m1, compute_dtype=torch.float32, fp32_names=[n for n, _ in m1.named_parameters()])
    o1 = fuse_optimizer_mt(make(list(m1.parameters())), arena)
    o2 = make(list(m2.parameters()))
    torch.manual_seed(0)
    for step in range(3):
        x = torch.randn(16, 1, 28, 28)
        for m, o in ((m1, o1), (m2, o2)):
            o.zero_grad()
            m.loss_fn(m(x), torch.arange(16) % 10).backward()
            o.step()
    for (k, a), b in zip(m1.state_dict().items(), m2.state_dict().values()):
        assert torch.allclose(a, b, atol=1e-5, rtol=1e-4), k


@pytest.mark.parametrize("opt_name", ["adam", "sgd"])
def test_channels_last_shadow_optimizer_matches_torch(opt_name):
    """Conv weights with a channels-last shadow: grads arrive NHWC-ordered, master/state stay OIHW, results == torch.optim."""
    from p2pfl_amd.learning.arena import ModuleArena
    from p2pfl_amd.learning.optim import fuse_optimizer_mt

    def net():
        torch.manual_seed(11)
        return torch.nn.Sequential(torch.nn.Conv2d(3, 8, 3, padding=1), torch.nn.ReLU(), torch.nn.Conv2d(8, 4, 1),
                                   torch.nn.Flatten(), torch.nn.Linear(4 * 6 * 6, 5))

    m1, m2 = net(), net()
    make = {
        "adam": lambda ps: torch.optim.Adam(ps, lr=1e-2, weight_decay=1e-3),
        "sgd": lambda ps: torch.optim.SGD(ps, lr=0.1, momentum=0.9, weight_decay=5e-4),
    }[opt_name]
    keep = [n for n, p in m1.named_parameters() if p.dim() < 2]
    arena = ModuleArena(m1, compute_dtype=torch.float32, fp32_names=keep, channels_last_names=["0.weight", "2.weight"])
    assert set(arena.shadow_cl) == {"0.weight"}  # 1x1 kernels need no permutation
    w0 = m1[0].weight
    assert w0.is_contiguous(memory_format=torch.channels_last) and not w0.is_contiguous()
    o1 = fuse_optimizer_mt(make(list(m1.parameters())), arena)
    assert o1.mt.grad_cl == [n == "0.weight" for n, _ in m1.named_parameters()]
    o2 = make(list(m2.parameters()))
    torch.manual_seed(0)
    for _ in range(3):
        x = torch.randn(8, 3, 6, 6).contiguous(memory_format=torch.channels_last)
        y = torch.arange(8) % 5
        for m, o in ((m1, o1), (m2, o2)):
            o.zero_grad()
            torch.nn.functional.cross_entropy(m(x), y).backward()
            o.step()
    for (k, a), b in zip(m1.state_dict().items(), m2.state_dict().values()):
        assert torch.allclose(a, b, atol=1e-5, rtol=1e-4), k
    master = arena.params["0.weight"]
    assert torch.equal(w0.detach(), master)  # shadow (NHWC memory) == master (OIHW) element-wise
    arena.params.flat.mul_(0.5)
    arena.refresh_shadow()
    assert torch.equal(w0.detach(), master)


def test_fedavg_running_sum_is_bitwise_equal_to_one_shot_for_any_arrival_order():
    """Models folded into the running sum as they arrive (any order, any
    interleaving with partial aggregations) give exactly the one-shot result."""
    import itertools
    import random

    import torch

    from p2pfl_amd.learning.aggregators.fedavg import FedAvg
    from p2pfl_amd.learning.arena import flatten

    names = ["n3", "n0", "n2", "n1", "n4"]
    rng = torch.Generator().manual_seed(0)
    models = {n: flatten({"w": torch.randn(37, 11, generator=rng), "b": torch.randn(5, generator=rng)}) for n in names}
    weights = {n: 100 + 17 * i for i, n in enumerate(names)}
    oneshot = FedAvg()
    oneshot.running_sum = False
    oneshot.set_nodes_to_aggregate(names)
    for n in names:
        oneshot.add_model(models[n], [n], weights[n])
    want = oneshot.wait_and_get_aggregation(timeout=1).flat.clone()
    orders = list(itertools.permutations(names))
    random.Random(1).shuffle(orders)
    folded_any = False
    for order in orders[:25]:
        agg = FedAvg()
        agg.set_nodes_to_aggregate(names)
        for n in order:
            agg.add_model(models[n], [n], weights[n])
            agg.get_partial_aggregation([])  # gossip asks for partial aggregates in between
            folded_any |= agg._run is not None and len(agg._run.keys) > 0
        got = agg.wait_and_get_aggregation(timeout=1).flat
        assert torch.equal(got, want), order
    assert folded_any
    ref = sum(models[n].flat * weights[n] for n in names) / sum(weights.values())
    torch.testing.assert_close(want, ref, rtol=1e-6, atol=1e-6)


def test_fedavg_partial_aggregates_are_exact_while_models_arrive_concurrently(monkeypatch):
    """Receive threads fold models into the running sum while gossip threads
    take partial aggregates: every partial must be the average of exactly the
    contributors it reports (a fold must never write an accumulator a reader
    already took -- ADVICE r3 high), and the final aggregate stays bitwise equal
    to the one-shot average."""
    import threading
    import time

    import torch

    from p2pfl_amd.learning.aggregators import fedavg as fedavg_mod
    from p2pfl_amd.learning.aggregators.fedavg import FedAvg
    from p2pfl_amd.learning.arena import flatten

    real_flatten = fedavg_mod.flatten

    def slow_flatten(*a, **k):  # widen the window between taking the sum and launching on it
        time.sleep(0.0005)
        return real_flatten(*a, **k)

    monkeypatch.setattr(fedavg_mod, "flatten", slow_flatten)
    names = [f"n{i}" for i in range(8)]
    rng = torch.Generator().manual_seed(3)
    models = {n: flatten({"w": torch.randn(64, 33, generator=rng), "b": torch.randn(9, generator=rng)}) for n in names}
    weights = {n: 50 + 13 * i for i, n in enumerate(names)}

    def expected(contribs):
        tot = sum(weights[c] for c in contribs)
        return sum(models[c].flat.double() * weights[c] for c in contribs) / tot

    oneshot = FedAvg()
    oneshot.running_sum = False
    oneshot.set_nodes_to_aggregate(names)
    for n in names:
        oneshot.add_model(models[n], [n], weights[n])
    want = oneshot.wait_and_get_aggregation(timeout=1).flat.clone()

    for trial in range(6):
        agg = FedAvg()
        agg.set_nodes_to_aggregate(names)
        errors = []
        stop = threading.Event()
        order = names[trial % 8:] + names[: trial % 8]

        def receiver(part):
            for n in part:
                agg.add_model(models[n], [n], weights[n])
                time.sleep(0.001)

        def gossiper(excl):
            while not stop.is_set():
                model, contribs, w = agg.get_partial_aggregation(excl)
                if model is None:
                    continue
                assert w == sum(weights[c] for c in contribs)
                got = (model.flat if hasattr(model, "flat") else model).double()
                if not torch.allclose(got, expected(contribs), rtol=1e-5, atol=1e-5):
                    errors.append(sorted(contribs))

        rx = [threading.Thread(target=receiver, args=(order[i::2],)) for i in range(2)]
        gx = [threading.Thread(target=gossiper, args=(ex,)) for ex in ([], [names[1]], [names[6]])]
        for t in gx + rx:
            t.start()
        for t in rx:
            t.join()
        stop.set()
        for t in gx:
            t.join()
        assert not errors, f"wrong partial aggregates for {errors[:3]}"
        assert torch.equal(agg.wait_and_get_aggregation(timeout=1).flat, want)


def test_check_finite_debug_mode_names_the_first_bad_tensor(monkeypatch):
    import pytest
    import torch

    from p2pfl_amd.learning.aggregators.fedavg import FedAvg
    from p2pfl_amd.learning.arena import flatten
    from p2pfl_amd.utils import finite

    monkeypatch.setattr(finite, "ENABLED", True)
    good = flatten({"w": torch.ones(8)})
    bad = flatten({"w": torch.tensor([1.0, float("nan")] + [0.0] * 6)})
    agg = FedAvg("nodeX")
    agg.set_nodes_to_aggregate(["a", "b"])
    agg.add_model(good, ["a"], 1)
    agg.add_model(bad, ["b"], 1)
    with pytest.raises(finite.NonFiniteError, match="FedAvg input.*key=b"):
        agg.wait_and_get_aggregation(timeout=1)
    finite.check("n", "fine", good)  # no error on finite data
