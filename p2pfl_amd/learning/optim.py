"""Whole-arena fused optimizers.

``torch.optim.Adam``/``SGD`` launch per-tensor (or per-group "foreach") kernels.
With parameters and gradients living in one flat arena, the entire update is a
single memory-bound HIP kernel (``csrc/optim.hip``): one read of
param/grad/state and one write, 16-byte vector accesses, fp32 math.  The
results match ``torch.optim`` to fp32 rounding (tested).

:func:`fuse_optimizer` inspects the optimizer a model's
``configure_optimizers`` returned and swaps in the fused equivalent when it is
a plain single-group Adam/AdamW/SGD over every parameter; anything else is
left to torch.
"""

from __future__ import annotations

from typing import Optional, Tuple

import torch

from p2pfl_amd import ops
from p2pfl_amd.learning.arena import ModuleArena


class _ArenaOptimizer:
    def __init__(self, arena: ModuleArena, lr: float, weight_decay: float) -> None:
        assert arena.grads is not None
        self.arena = arena
        self.lr = lr
        self.weight_decay = weight_decay
        self.t = 0
        # Buffers (BatchNorm running stats, mirrored integer counters) share the
        # arena with the parameters but must not be touched by the update
        # (weight decay would shrink them): their elements are saved before and
        # restored after each fused step -- a few KB against a full-arena kernel.
        params = set(arena.param_names)
        lay = arena.layout
        idx = [
            torch.arange(off, off + n, dtype=torch.int64)
            for name, off, n in zip(lay.names, lay.offsets, lay.sizes())
            if name not in params and n > 0
        ]
        self._buf_idx = torch.cat(idx).to(arena.flat.device) if idx else None

    def _step_keep_buffers(self, fn) -> None:
        saved = self.arena.flat.index_select(0, self._buf_idx) if self._buf_idx is not None else None
        fn()
        if saved is not None:
            self.arena.flat.index_copy_(0, self._buf_idx, saved)

    def zero_grad(self, set_to_none: bool = False) -> None:
        assert self.arena.grads is not None
        self.arena.grads.zero_()

    def _grads(self) -> torch.Tensor:
        if not self.arena.grads_bound():
            self.arena.rebind_grads()
        assert self.arena.grads is not None
        return self.arena.grads


class ArenaAdam(_ArenaOptimizer):
    def __init__(
        self,
        arena: ModuleArena,
        lr: float = 1e-3,
        betas=(0.9, 0.999),
        eps: float = 1e-8,
        weight_decay: float = 0.0,
        decoupled: bool = False,
    ) -> None:
        super().__init__(arena, lr, weight_decay)
        self.beta1, self.beta2 = betas
        self.eps = eps
        self.decoupled = decoupled
        self.m = torch.zeros_like(arena.flat)
        self.v = torch.zeros_like(arena.flat)

    def step(self) -> None:
        self.t += 1
        self._step_keep_buffers(
            lambda: ops.adam_step(
                self.arena.flat,
                self._grads(),
                self.m,
                self.v,
                lr=self.lr,
                beta1=self.beta1,
                beta2=self.beta2,
                eps=self.eps,
                weight_decay=self.weight_decay,
                step=self.t,
                decoupled=self.decoupled,
            )
        )


class ArenaSGD(_ArenaOptimizer):
    def __init__(
        self,
        arena: ModuleArena,
        lr: float = 1e-2,
        momentum: float = 0.0,
        dampening: float = 0.0,
        weight_decay: float = 0.0,
        nesterov: bool = False,
    ) -> None:
        super().__init__(arena, lr, weight_decay)
        self.momentum, self.dampening, self.nesterov = momentum, dampening, nesterov
        self.buf: Optional[torch.Tensor] = torch.zeros_like(arena.flat) if momentum != 0 else None

    def step(self) -> None:
        self.t += 1
        self._step_keep_buffers(
            lambda: ops.sgd_step(
                self.arena.flat,
                self._grads(),
                self.buf,
                lr=self.lr,
                momentum=self.momentum,
                dampening=self.dampening,
                weight_decay=self.weight_decay,
                nesterov=self.nesterov,
                first_step=self.t == 1,
            )
        )


def fuse_optimizer(opt: torch.optim.Optimizer, arena: ModuleArena):
    """Return a fused arena optimizer equivalent to ``opt``, or None."""
    if len(opt.param_groups) != 1 or arena.grads is None:
        return None
    g = opt.param_groups[0]
    params = {id(p) for p in g["params"]}
    if params != {id(p) for p in arena.module.parameters()}:
        return None
    if g.get("maximize") or g.get("differentiable"):
        return None
    lr = float(g["lr"]) if not isinstance(g["lr"], torch.Tensor) else float(g["lr"].item())
    if type(opt) is torch.optim.Adam and not g.get("amsgrad"):
        return ArenaAdam(arena, lr, tuple(g["betas"]), g["eps"], g["weight_decay"], decoupled=False)
    if type(opt) is torch.optim.AdamW and not g.get("amsgrad"):
        return ArenaAdam(arena, lr, tuple(g["betas"]), g["eps"], g["weight_decay"], decoupled=True)
    if type(opt) is torch.optim.SGD:
        return ArenaSGD(arena, lr, g["momentum"], g["dampening"], g["weight_decay"], g["nesterov"])
    return None


# ----------------------------------------------------------------------------
# Multi-tensor optimizers for mixed-precision arenas (ModuleArena(compute_dtype=...))
# ----------------------------------------------------------------------------
MT_CHUNK = 4096  # csrc/kernels.h kMTChunk
MT_MAX_CL = 4608  # csrc/kernels.h kMTMaxCL


def mt_layout(table, dev) -> Tuple[torch.Tensor, torch.Tensor]:
    """Device tables of the multi-tensor kernels for ``table`` = [(offset, numel,
    flags)]: ``tens`` int64 [T, 4] = (offset, numel, flags, elements per
    block) and ``chunks`` int32 [C, 2] = (tensor, first element), one GPU
    block per chunk.  A channels-last tensor (flags bit 2) whose output-channel
    slab (I x kh x kw elements, I % 4 == 0) fits csrc/optim.hip's LDS stage
    gets chunks of whole slabs, which the kernel reads and writes contiguously;
    every other tensor 4096-element chunks."""
    rows, chunks = [], []
    for t, (off, n, flags) in enumerate(table):
        chunk = MT_CHUNK
        if flags & 4:
            i, hw = (flags >> 8) & 0xFFFFFF, (flags >> 32) & 0xFFFFFF
            per_o = i * hw
            if hw > 1 and i % 4 == 0 and per_o <= MT_MAX_CL:
                chunk = per_o * (MT_MAX_CL // per_o)
        rows.append((off, n, flags, chunk))
        chunks.extend((t, c) for c in range(0, n, chunk))
    if any(c >= 2**31 for _, c in chunks):
        raise ValueError("multi-tensor chunk offset exceeds int32")
    tens = torch.tensor(rows, dtype=torch.int64, device=dev).reshape(-1, 4)
    return tens, torch.tensor(chunks, dtype=torch.int32, device=dev).reshape(-1, 2)


class MTTables:
    """Static per-tensor and per-chunk tables for the multi-tensor kernels.

    ``table`` = [(arena offset, numel, flags)] with flags bit 0 = bf16
    gradient, bit 1 = write the bf16 shadow, bit 2 = gradient and shadow are
    channels-last (O, kh, kw, I) with I in bits 8..31 and kh*kw in bits
    32..55 (the fp32 state stays OIHW); ``tens`` / ``chunks``: the device
    tables of :func:`mt_layout`.
    """

    CHUNK = MT_CHUNK

    def __init__(self, arena: ModuleArena) -> None:
        lay = arena.layout
        shadow = set(arena.shadow_names)
        self.params = [p for _, p in arena.module.named_parameters()]
        names = [n for n, _ in arena.module.named_parameters()]
        self.table = []
        for t, (name, p) in enumerate(zip(names, self.params)):
            off = lay.offsets[lay.names.index(name)]
            flags = (1 if p.dtype == torch.bfloat16 else 0) | (2 if name in shadow else 0)
            if name in arena.shadow_cl:
                o, i, kh, kw = arena.shadow_cl[name][1]
                flags |= 4 | (i << 8) | ((kh * kw) << 32)
            self.table.append((off, p.numel(), flags))
        dev = arena.flat.device
        self.numels = [n for _, n, _ in self.table]
        self.grad_bf16 = [bool(f & 1) for _, _, f in self.table]
        self.grad_cl = [bool(f & 4) for _, _, f in self.table]
        self.tens, self.chunks = mt_layout(self.table, dev)

    def grads(self):
        return [p.grad for p in self.params]

    def fill_grad_table(self, gtab: torch.Tensor) -> None:
        """Write the current gradients' addresses into the persistent device table ``gtab``."""
        for p, cl in zip(self.params, self.grad_cl):
            if p.grad is not None and not p.grad.is_contiguous(memory_format=torch.channels_last if cl else torch.contiguous_format):
                raise RuntimeError(f"gradient of shape {tuple(p.grad.shape)} is not in its parameter's layout")
        ptrs = [p.grad.data_ptr() if p.grad is not None else 0 for p in self.params]
        gtab.copy_(torch.tensor(ptrs, dtype=torch.int64))


class _MTOptimizer:
    """Base of the multi-tensor optimizers.

    ``step()`` is the eager path (gradient addresses gathered per call);
    ``step_graph(gtab)`` reads them from a persistent device table and keeps
    every step-dependent scalar on the device, so it can be captured once in
    a HIP graph and replayed (:mod:`p2pfl_amd.learning.step_graph`).
    ``reset()`` returns the optimizer to its freshly-constructed state while
    keeping its buffers' addresses (a captured graph stays valid).
    """

    def __init__(self, arena: ModuleArena, lr: float, weight_decay: float) -> None:
        self.arena = arena
        self.lr = lr
        self.weight_decay = weight_decay
        self.t = 0
        self.mt = MTTables(arena)

    def config(self) -> tuple:
        return (type(self).__name__, self.lr, self.weight_decay)

    def state_tensors(self) -> list:
        return []

    def reset(self) -> None:
        self.t = 0
        for t in self.state_tensors():
            t.zero_()

    def graph_first_step_ok(self) -> bool:
        """Whether ``step_graph`` on freshly reset state equals the eager first step
        (so a fit can replay its captured graph from step 0)."""
        return True

    def zero_grad(self, set_to_none: bool = True) -> None:
        # always None: autograd then hands over each new gradient without a
        # zero-fill + accumulate kernel per parameter
        for p in self.mt.params:
            p.grad = None


class MTAdam(_MTOptimizer):
    def __init__(self, arena, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, decoupled=False) -> None:
        super().__init__(arena, lr, weight_decay)
        self.beta1, self.beta2 = betas
        self.eps = eps
        self.decoupled = decoupled
        self.m = torch.zeros_like(arena.flat)
        self.v = torch.zeros_like(arena.flat)
        self.t_dev = torch.zeros(1, dtype=torch.int32, device=arena.flat.device)

    def config(self) -> tuple:
        return super().config() + (self.beta1, self.beta2, self.eps, self.decoupled)

    def state_tensors(self) -> list:
        return [self.m, self.v, self.t_dev]

    def step(self) -> None:
        self.t += 1
        ops.adam_mt_step(
            self.arena.flat, self.m, self.v, self.mt.grads(), self.mt,
            lr=self.lr, beta1=self.beta1, beta2=self.beta2, eps=self.eps,
            weight_decay=self.weight_decay, step=self.t, decoupled=self.decoupled, p_bf16=self.arena.shadow,
        )
        if self.arena.flat.is_cuda:
            self.t_dev.fill_(self.t)

    def step_graph(self, gtab: torch.Tensor) -> None:
        """Graph-capturable step: t_dev += 1 on the device, bias corrections from it."""
        self.t_dev.add_(1)
        ops.adam_mt_step(
            self.arena.flat, self.m, self.v, [], self.mt,
            lr=self.lr, beta1=self.beta1, beta2=self.beta2, eps=self.eps,
            weight_decay=self.weight_decay, step=1, decoupled=self.decoupled, p_bf16=self.arena.shadow,
            gtab=gtab, t_dev=self.t_dev,
        )


class MTSGD(_MTOptimizer):
    def __init__(self, arena, lr=1e-2, momentum=0.0, dampening=0.0, weight_decay=0.0, nesterov=False) -> None:
        super().__init__(arena, lr, weight_decay)
        self.momentum, self.dampening, self.nesterov = momentum, dampening, nesterov
        self.buf: Optional[torch.Tensor] = torch.zeros_like(arena.flat) if momentum != 0 else None

    def config(self) -> tuple:
        return super().config() + (self.momentum, self.dampening, self.nesterov)

    def state_tensors(self) -> list:
        return [self.buf] if self.buf is not None else []

    def step(self) -> None:
        self.t += 1
        ops.sgd_mt_step(
            self.arena.flat, self.buf, self.mt.grads(), self.mt,
            lr=self.lr, momentum=self.momentum, dampening=self.dampening, weight_decay=self.weight_decay,
            nesterov=self.nesterov, first_step=self.t == 1, p_bf16=self.arena.shadow,
        )

    def graph_first_step_ok(self) -> bool:
        # eager step 1 seeds buf = g; the graph step computes buf = m * buf + (1 - dampening) g,
        # which on the zeroed buffer of a reset optimizer is exactly g when dampening == 0
        return self.buf is None or self.dampening == 0

    def step_graph(self, gtab: torch.Tensor) -> None:
        """Graph-capturable step (momentum buffer already seeded, or zero with dampening 0)."""
        ops.sgd_mt_step(
            self.arena.flat, self.buf, [], self.mt,
            lr=self.lr, momentum=self.momentum, dampening=self.dampening, weight_decay=self.weight_decay,
            nesterov=self.nesterov, first_step=False, p_bf16=self.arena.shadow, gtab=gtab,
        )


def fusable(opt: torch.optim.Optimizer, module: torch.nn.Module) -> bool:
    """True if ``opt`` is a plain single-group Adam/AdamW/SGD over all of ``module``'s parameters."""
    if len(opt.param_groups) != 1:
        return False
    g = opt.param_groups[0]
    if {id(p) for p in g["params"]} != {id(p) for p in module.parameters()}:
        return False
    if g.get("maximize") or g.get("differentiable") or g.get("amsgrad"):
        return False
    return type(opt) in (torch.optim.Adam, torch.optim.AdamW, torch.optim.SGD)


def fuse_optimizer_mt(opt: torch.optim.Optimizer, arena: ModuleArena):
    """Multi-tensor equivalent of ``opt`` for a mixed-precision arena, or None."""
    if not fusable(opt, arena.module):
        return None
    g = opt.param_groups[0]
    lr = float(g["lr"]) if not isinstance(g["lr"], torch.Tensor) else float(g["lr"].item())
    if type(opt) is torch.optim.SGD:
        return MTSGD(arena, lr, g["momentum"], g["dampening"], g["weight_decay"], g["nesterov"])
    return MTAdam(arena, lr, tuple(g["betas"]), g["eps"], g["weight_decay"], decoupled=type(opt) is torch.optim.AdamW)
