"""HIP-graph-replayed training steps == the eager loop (MI355X only).

Eager ResNet training on MIOpen is itself not bitwise reproducible (two
eager learners from the same seed drift apart by O(0.1-1) in the largest
weights over a round), so ResNet is checked for equal bookkeeping and
equivalent training; models whose eager step IS reproducible (linear layers,
ViT) are compared tensor by tensor.
"""

from __future__ import annotations

import pytest
import torch
from torch import nn

from p2pfl_amd.models.base import FLModule

pytestmark = pytest.mark.gpu


class _SGDNet(FLModule):
    """Linear/ReLU net with SGD+momentum+weight decay (the ResNet optimizer, deterministic kernels)."""

    def __init__(self) -> None:
        super().__init__()
        torch.manual_seed(0)
        self.net = nn.Sequential(nn.Flatten(), nn.Linear(3 * 32 * 32, 256), nn.ReLU(), nn.Linear(256, 10))

    def forward(self, x):
        return self.net(x.float() if x.dtype == torch.uint8 else x)

    def configure_optimizers(self):
        return torch.optim.SGD(self.parameters(), lr=0.05, momentum=0.9, weight_decay=5e-4)


def _cifar():
    from p2pfl_amd.data import Cifar10FederatedDM

    return Cifar10FederatedDM(sub_id=0, number_sub=200, batch_size=32)


def _pair(make):
    from p2pfl_amd.learning.torch_learner import TorchLearner

    out = []
    for graphs in (False, True):
        torch.manual_seed(0)
        out.append(TorchLearner(make(), _cifar(), "p", 1, device=torch.device("cuda", 0), use_step_graphs=graphs))
    return out


@pytest.mark.parametrize("name", ["sgd_net", "vit_tiny"])
def test_step_graph_matches_eager(name):
    from p2pfl_amd.models.vit import ViT_Tiny

    make = {"sgd_net": _SGDNet, "vit_tiny": lambda: ViT_Tiny(seed=0)}[name]
    eager, graph = _pair(make)
    assert graph.mixed and eager.mixed
    assert len(graph.data.train_dataloader().dataset) > 2 * 32  # several full batches replayed (the first too: dampening 0)
    for _round in range(2):  # the second fit reuses the captured graph after an optimizer reset
        eager.fit()
        graph.fit()
        torch.cuda.synchronize()
        for (k, x), y in zip(eager.get_parameters().items(), graph.get_parameters().values()):
            torch.testing.assert_close(y, x, atol=1e-2, rtol=1e-2, msg=lambda m, k=k: f"{name} {k}: {m}")
    assert graph._step_graph is not None and graph._step_graph.graph is not None
    n_train = len(graph.data.train_dataloader().dataset)
    if n_train % 32 > 1:  # the short last batch replays a graph of its own size
        assert set(graph._tail_graphs) == {n_train % 32}
    assert graph._step == eager._step
    # evaluation passes replay a captured forward graph: same metrics as the eager loop
    graph.set_parameters(eager.get_parameters())
    ev_e, ev_g = eager.evaluate(), graph.evaluate()
    assert set(ev_e) == set(ev_g) == {"test_loss", "test_metric"}
    assert graph._eval_graphs and all(g.graph is not None for g in graph._eval_graphs.values())
    for k in ev_e:
        assert abs(ev_e[k] - ev_g[k]) <= 1e-3 + 1e-3 * abs(ev_e[k]), (k, ev_e, ev_g)


def _train_mode_loss(ln) -> float:
    """Mean train-mode (batch-statistics) loss over the local train shard, on a copy of the model."""
    import copy

    m = copy.deepcopy(ln.model).train()
    ld = ln.data.train_dataloader()
    tot, n = 0.0, 0
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        for s in range(0, len(ld.dataset) - 31, 32):
            idx = torch.arange(s, s + 32, device=ld.x.device)
            x = ld.x.index_select(0, idx).float().div_(255.0)
            tot += float(torch.nn.functional.cross_entropy(m(x).float(), ld.y.index_select(0, idx))) * 32
            n += 32
    return tot / n


def test_step_graph_resnet18_trains_like_eager():
    from p2pfl_amd.models.resnet import ResNet18

    eager, graph = _pair(lambda: ResNet18(seed=0, lr_rate=0.01))
    first = _train_mode_loss(graph)
    for _round in range(3):
        eager.fit()
        graph.fit()
    torch.cuda.synchronize()
    assert graph._step_graph is not None and graph._step == eager._step
    sd_e, sd_g = eager.model.state_dict(), graph.model.state_dict()
    for k in sd_e:
        if "num_batches_tracked" in k:
            assert int(sd_e[k]) == int(sd_g[k]) == eager._step, k
        else:
            assert torch.isfinite(sd_g[k]).all(), k
    le, lg = _train_mode_loss(eager), _train_mode_loss(graph)
    # both fit the shard; the graph run lands where the eager one does
    assert lg < first and le < first, (first, le, lg)
    assert abs(le - lg) < 0.5 * max(le, lg, 0.1), (first, le, lg)


def test_resnet_channels_last_weight_shadows():
    """ResNet spatial conv weights are channels-last bf16 shadows; MIOpen hands back channels-last grads, and
    after graph-replayed steps every shadow equals its fp32 OIHW master rounded to bf16."""
    from p2pfl_amd.learning.torch_learner import TorchLearner
    from p2pfl_amd.models.resnet import ResNet18

    torch.manual_seed(0)
    ln = TorchLearner(ResNet18(seed=0, lr_rate=0.01), _cifar(), "p", 1, device=torch.device("cuda", 0), use_step_graphs=True)
    arena = ln.arena
    named = dict(ln.model.named_parameters())
    assert arena.shadow_cl and all(named[n].is_contiguous(memory_format=torch.channels_last) for n in arena.shadow_cl)
    # one eager backward: the conv weight grads arrive in the weights' own layout (no relayout copy)
    x, y = next(iter(ln.data.train_dataloader()))
    with torch.autocast("cuda", dtype=torch.bfloat16):
        torch.nn.functional.cross_entropy(ln.model(x.cuda()), y.cuda()).backward()
    for n in arena.shadow_cl:
        g = named[n].grad
        assert g is not None and g.dtype == torch.bfloat16 and g.is_contiguous(memory_format=torch.channels_last), n
        named[n].grad = None
    ln.model.zero_grad(set_to_none=True)
    ln.fit()
    torch.cuda.synchronize()
    for n in arena.shadow_names:
        assert torch.equal(named[n].detach(), arena.params[n].to(torch.bfloat16)), n


def test_eval_graph_batches_several_loader_batches():
    """Captured evaluation steps take Settings.EVAL_BATCH_FACTOR loader batches at once
    (ragged tail eager): same metrics as the eager per-batch loop."""
    from p2pfl_amd.data import Cifar10FederatedDM
    from p2pfl_amd.learning.torch_learner import TorchLearner
    from p2pfl_amd.models.vit import ViT_Tiny

    out = []
    for graphs in (False, True):
        torch.manual_seed(0)
        dm = Cifar10FederatedDM(sub_id=0, number_sub=30, batch_size=32)
        ln = TorchLearner(ViT_Tiny(seed=0), dm, "p", 1, device=torch.device("cuda", 0), use_step_graphs=graphs)
        out.append((ln, ln.evaluate()))
    (eager, ev_e), (graph, ev_g) = out
    ld = graph.data.test_dataloader()
    n, B = len(ld.dataset), graph._eval_batch(ld)
    assert B > 32 and n % B and n > B, (n, B)  # several multi-batch replays plus a remainder
    assert {g.B for g in graph._eval_graphs.values()} == {B, n % B}  # full batches + the remainder's graph
    for k in ev_e:
        assert abs(ev_e[k] - ev_g[k]) <= 2e-3 + 2e-3 * abs(ev_e[k]), (k, ev_e, ev_g)
