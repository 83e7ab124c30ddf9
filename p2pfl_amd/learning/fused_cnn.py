"""MI355X-native training engine for the reference MNIST CNN.

:class:`FusedCNNEngine` runs the whole training step of
:class:`~p2pfl_amd.models.cnn.CNN` through the hand-written HIP kernels of
``csrc/cnn_fwd.hip`` / ``csrc/cnn_bwd.hip`` (pipeline in ``csrc/cnn.h``): no
autograd, no per-layer optimizer launches, bf16 MFMA compute with fp32 master
weights and fp32 Adam state kept in the model's flat arena.  A whole epoch
(every step, with its data indices) is captured ONCE as a HIP graph and then
replayed, so a step costs 8 kernel boundaries and zero host work.

:class:`FusedCNNLearner` is the :class:`~p2pfl_amd.learning.learner.NodeLearner`
on top of it (same parameter/wire behaviour as ``TorchLearner``, so fused and
torch peers interoperate).  It is selected automatically for ``CNN`` models on
a GPU by :func:`auto_learner`.
"""

from __future__ import annotations

import collections
import math
import os
import threading
import time
from typing import Any, Dict, List, Optional, Tuple

import torch

from p2pfl_amd import ops
from p2pfl_amd.learning.arena import FlatParams, ModuleArena
from p2pfl_amd.learning.host_completion import HostCompletions
from p2pfl_amd.learning.torch_learner import TorchLearner
from p2pfl_amd.management.logger import logger
from p2pfl_amd.utils.lockcheck import make_lock, make_rlock
from p2pfl_amd.utils.streams import private_stream

# Several learners (virtual peers on one GPU, each on its own node thread)
# may capture epoch graphs concurrently: captures are serialised process-wide
# and run in thread-local capture mode, so the other peers' kernels and
# allocations on their own threads stay legal while one peer captures.
_CAPTURE_LOCK = make_lock("FusedCNN._CAPTURE_LOCK")
# fits the host may run ahead of the device (P2PFL_FIT_RUN_AHEAD; 1 = the round-4 bound)
RUN_AHEAD = max(1, int(os.environ.get("P2PFL_FIT_RUN_AHEAD", "2")))

# conv_adam folded into the FC1 Adam launch (P2PFL_CNN_MERGED_ADAM=0: separate launches)
_MERGED_ADAM = os.environ.get("P2PFL_CNN_MERGED_ADAM", "1") != "0"
# dA1 routing reads the row-major W1 shadow through LDS transpose reads (no
# W1^T shadow, 12.8 MB less written per step by the FC1 Adam stream); "0"
# selects the W1^T-shadow kernel.
_ROUTE_RM = os.environ.get("P2PFL_CNN_ROUTE_RM", "1") != "0"
# dA1 routing split over 2 K-slices per feature tile (196 workgroups instead of
# 98, the last slice to arrive reduces; csrc/cnn_bwd.hip route_rm_kernel).  Off:
# measured 17.2 us vs 7.5 us unsplit (scripts/kbench.py, MI355X, round 4) -- the
# cross-CU hand-off costs more than the halved per-workgroup stream saves.
_ROUTE_SPLIT = os.environ.get("P2PFL_CNN_ROUTE_SPLIT", "0") == "1"
_EVAL_LOW = os.environ.get("P2PFL_EVAL_STREAM_LOW", "1") != "0"
# evaluation passes on their own stream beside the next training ("1") or in line
# on the learner's stream ("0", default; "auto": beside it when the learner has a
# stream of its own).  In line: no stream hand-offs between the epoch and its
# validation pass (1-peer round: in line 6.65 vs 7.23 ms, profiles/r5_handoff_probe.md).
_EVAL_SIDE = os.environ.get("P2PFL_EVAL_SIDE_STREAM", "0")
# conv1 + conv2 in one launch (csrc/cnn_fwd.hip conv12_fwd_kernel: each pooled-row block
# recomputes the P1 rows its conv2 reads in LDS; no P1 round trip, one launch less).
# Opt-in (P2PFL_CNN_CONV12=1): measured slower, 16.3 us vs 4.6 + 6.0 us for the two
# kernels and 7.27 vs 6.66 ms per headline round (scripts/kbench.py, MI355X, round 6) --
# the 3x conv1 VALU work of the recomputed halo rows sits in front of conv2 in every block.
_CONV12 = os.environ.get("P2PFL_CNN_CONV12", "0") == "1"
# The next step's conv1 + conv2 inside this step's last launch, beside the FC1 Adam
# stream (csrc/cnn_bwd.hip fc1_conv_adam_fwd_kernel; A1 double-buffered by step
# parity).  Opt-in (P2PFL_CNN_FWD_IN_ADAM=1), measured slower on MI355X (round 6,
# rocprofv3 of bench.py): the launch takes 66-72 us against 28.8 + 4.6 + 6.0 us for
# the three kernels, 8.6-9.4 vs 6.66 ms per headline round -- the convolutions'
# device-coherent (sc1) reads of the freshly updated weights and of P1 miss every
# cache, and their waits hold CU slots; bitwise-equal results
# (tests/test_gpu_fused_cnn.py::test_next_forward_inside_the_adam_launch_is_bitwise_equal).
_FWD_IN_ADAM = os.environ.get("P2PFL_CNN_FWD_IN_ADAM", "0") == "1"
_NAMES = ("conv1.weight", "conv1.bias", "conv2.weight", "conv2.bias", "l1.weight", "l1.bias", "l2.weight", "l2.bias")
FEAT, HID = 3136, 2048


class FusedCNNEngine:
    """Kernel-level forward/backward/Adam for the MNIST CNN on one GPU."""

    def __init__(
        self,
        model: torch.nn.Module,
        device: Optional[torch.device] = None,
        lr: float = 1e-3,
        betas: Tuple[float, float] = (0.9, 0.999),
        eps: float = 1e-8,
        weight_decay: float = 0.0,
        mrows: int = 32,
        arena: Optional[ModuleArena] = None,
        split_fc1: Optional[int] = None,
    ) -> None:
        self.C = ops.ext().cnn
        self.C.init()
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        model.to(self.device)
        self.arena = arena if arena is not None else ModuleArena(model, device=self.device)
        lay = self.arena.layout
        if tuple(lay.names) != _NAMES:
            raise ValueError(f"FusedCNNEngine needs the reference CNN layout {_NAMES}, got {lay.names}")
        shapes = dict(zip(lay.names, lay.shapes))
        if shapes["conv1.weight"] != (32, 1, 5, 5) or shapes["l2.weight"][1] != HID or shapes["l2.weight"][0] != 10:
            raise ValueError("unsupported CNN configuration (needs 1x28x28 input, 10 classes)")
        self.off: List[int] = [int(o) for o in lay.offsets]
        self.lr, self.betas, self.eps, self.wd = lr, betas, eps, weight_decay
        self.mrows = mrows
        # K-slices of the FC1 GEMM (gemm_skinny: 64 column tiles x S1 workgroups); the
        # head reads the S1 fp32 partial rows of its sample, so fewer slices mean fewer
        # bytes for the head's 32 workgroups (P2PFL_CNN_FC1_SPLITS overrides)
        self.S1 = int(split_fc1 if split_fc1 is not None else os.environ.get("P2PFL_CNN_FC1_SPLITS", "7"))
        if not 1 <= self.S1 <= 49:
            raise ValueError(f"FC1 split count {self.S1} outside [1, 49]")
        dev, bf = self.device, torch.bfloat16
        z = lambda *s, dt=torch.float32: torch.zeros(*s, dtype=dt, device=dev)  # noqa: E731
        n = self.arena.flat.numel()
        # Adam moments and the device step base share ONE buffer, so the per-fit
        # optimizer reset (reference quirk Q23) is a single fill launch between
        # two epochs instead of three (v starts 16-byte aligned for the float4 streams)
        npad = (n + 3) // 4 * 4
        self._opt_state = z(2 * npad + 4)
        self.m, self.v = self._opt_state[:n], self._opt_state[npad:npad + n]
        self.adam_t = self._opt_state[2 * npad:2 * npad + 1].view(torch.int32)
        # bf16 weight shadows in kernel-friendly layouts
        self.w2r, self.w2q = z(51200, dt=bf), z(51200, dt=bf)
        self.route_rm = _ROUTE_RM
        self.w1bf = z(HID * FEAT, dt=bf)
        self.w1tbf = None if self.route_rm else z(HID * FEAT, dt=bf)
        # bf16 FC2 weight read by the head (half the bytes of the fp32 master per
        # head workgroup); refreshed by the merged Adam launch's FC2 blocks, so only
        # kept on that path
        self.w2bf = z(10 * HID, dt=bf) if _MERGED_ADAM else None
        # activations / workspaces (sized for mrows samples)
        M = mrows
        self.p1, self.am1 = z(M * 196 * 32, dt=bf), z(M * 196 * 32, dt=torch.uint8)
        # kx-shifted planar P1 copies for conv2_wgrad; padding cells stay zero
        self.p1s = z(M * 5 * 32 * 18 * 16, dt=bf)
        # A1 by step parity: a launch that runs the next step's conv2 (fc1_conv_adam_fwd)
        # writes the other buffer while its FC1 weight gradient reads the current one
        self._a1s = (z(M * FEAT, dt=bf), z(M * FEAT, dt=bf))
        self._par = 0
        self.am2 = z(M * FEAT, dt=torch.uint8)
        self._fwd_sync = z(4, dt=torch.int32)  # fc1_conv_adam_fwd tickets (self-resetting) + timeout flag
        self.slabs1 = z(self.S1 * M * HID)
        self.H, self.dH = z(M * HID, dt=bf), z(M * HID, dt=bf)
        self.dlogits = z(M * 10)
        # dC2 map written by route_fc2 (its padding columns stay zero from here on)
        self.dc2m, self.gb = z(M * 64 * 224, dt=bf), z(M * FEAT)
        self.wslab1, self.wslab2 = z(M * 7 * 832), z(self.C.wgrad_groups(M) * 51200)
        self.stats = z(2)
        # split-K partials + tickets of the routing kernel (tickets return to zero after every launch)
        split = self.route_rm and _ROUTE_SPLIT
        self.route_ws = z(98 * 2 * M * 32) if split else None
        self.route_ctr = z(98, dt=torch.int32) if split else None
        self.gdump: Optional[torch.Tensor] = None
        self.pack_shadows()

    # -- parameters -------------------------------------------------------
    @property
    def a1(self) -> torch.Tensor:
        """The pooled conv2 output of the current step (parity buffer)."""
        return self._a1s[self._par]

    @property
    def params(self) -> torch.Tensor:
        return self.arena.flat

    @property
    def w1_route(self) -> torch.Tensor:
        """The W1 operand of the dA1 routing kernel (row-major W1, or the W1^T shadow)."""
        return self.w1bf if self.route_rm else self.w1tbf

    def pack_shadows(self) -> None:
        """Refresh the bf16 weight copies after the fp32 parameters changed externally."""
        self.C.pack_shadows(self.params, self.off, self.w2r, self.w2q, self.w1bf, self.w1tbf, self.w2bf)

    def reset_optimizer(self) -> None:
        self._opt_state.zero_()  # m, v and the step base (int 0 = float 0 bits)

    # -- kernels ------------------------------------------------------------
    def _adam(self):
        return (self.lr, self.betas[0], self.betas[1], self.eps, self.wd)

    def forward(self, x: torch.Tensor, labels: torch.Tensor, idx: Optional[torch.Tensor], B: int, stats: torch.Tensor, train: bool,
                convs: bool = True) -> None:
        """The forward pass (``convs`` False: conv1 / conv2 already ran -- inside the
        previous step's last launch -- only the FC1 GEMM and the head remain)."""
        C, M = self.C, self.mrows
        if not convs:
            pass
        elif _CONV12:
            C.conv12_fwd(x, idx, self.params, self.off, self.w2r, None, self.am1, self.p1s if train else None, self.a1,
                         self.am2, B, M)
        else:
            C.conv1_fwd(x, idx, self.params, self.off, self.p1, self.am1, self.p1s if train else None, B)
            C.conv2_fwd(self.p1, self.w2r, self.params, self.off, self.a1, self.am2, B, M)
        C.gemm_skinny(self.a1, self.w1bf, self.slabs1, M, HID, FEAT, self.S1)
        C.head(self.slabs1, self.S1, M, self.params, self.off, labels, idx, B, train, self.H, self.dH, self.dlogits, stats,
               self.w2bf)

    def train_step_async(
        self, x: torch.Tensor, labels: torch.Tensor, idx: Optional[torch.Tensor], B: int, stats: torch.Tensor, t_off: int,
        nxt: Optional[Tuple[Optional[torch.Tensor], int]] = None, fwd_done: bool = False,
    ) -> None:
        """Enqueue one training step (no host sync; graph-capturable).

        Adam uses step ``t = adam_t[0] + t_off`` (base on the device, offset baked
        into the launch), so a captured epoch needs no per-step counter kernel.

        All kernels run on one stream.  Running the HBM-bound FC updates on a
        side stream (overlapping the latency-bound conv backward) was measured
        on MI355X at 146 us/step vs 119 us serial: each cross-queue edge of a
        HIP graph costs more than the overlap saves at this granularity.
        The FC2 gradient + Adam blocks ride in that same launch rather than in
        route_fc2's: sharing route_fc2's launch they did not overlap with the
        dA1 blocks (11.8 us together vs 6.7 + 7.4 us alone, scripts/kbench.py).
        Fusing route_fc2 and fc1_wgrad_adam horizontally into one launch
        (route blocks first, then the FC1 Adam stream; W1^T ping-ponged so the
        two roles need no ordering) was also measured: 50.8 us vs 12.6 + 33.8 us
        separately. The 512-thread blocks and the union LDS lower the FC1
        role's occupancy more than the overlap hides.  The conv-parameter Adam
        (256-thread blocks, 4 KB of LDS) does share the FC1 launch
        (``fc1_conv_adam``): it adds nothing to the FC1 role's footprint.
        """
        if B > self.mrows:
            raise ValueError(f"batch {B} > engine capacity {self.mrows}")
        C, M, a = self.C, self.mrows, self._adam()
        self.forward(x, labels, idx, B, stats, True, convs=not fwd_done)
        if _MERGED_ADAM:
            # dA1 routing alone, the conv backward, then ONE launch for the
            # FC2 and conv-parameter Adam (latency-bound) and the FC1 wgrad +
            # Adam stream (HBM-bound)
            C.route_fc2(self.dH, self.w1_route, self.am2, M, B, self.dc2m, self.gb, self.dlogits, self.H,
                        self.params, self.m, self.v, self.gdump, self.off, self.adam_t, t_off, *a, False, self.route_rm,
                        self.route_ws, self.route_ctr)
            C.conv2_bwd(self.dc2m, self.p1s, self.am1, self.w2q, x, idx, self.wslab1, self.wslab2, B)
            if nxt is not None and M <= 64:
                # ... with the next step's conv1 + conv2 (nxt = its row indices and batch) in the
                # same launch; the next step then passes fwd_done
                idx_n, Bn = nxt
                C.fc1_conv_adam_fwd(self.dH, self.a1, M, self.wslab1, self.wslab2, self.gb, B, self.params, self.m,
                                    self.v, self.gdump, self.w1bf, self.w1tbf, self.w2r, self.w2q, self.off, self.adam_t,
                                    t_off, *a, self.dlogits, self.H, self.w2bf, x, idx_n, self.p1, self.am1, self.p1s,
                                    self._a1s[1 - self._par], self.am2, Bn, self._fwd_sync)
                self._par ^= 1
                return
            C.fc1_conv_adam(self.dH, self.a1, M, self.wslab1, self.wslab2, self.gb, B, self.params, self.m, self.v,
                            self.gdump, self.w1bf, self.w1tbf, self.w2r, self.w2q, self.off, self.adam_t, t_off, *a,
                            self.dlogits, self.H, self.w2bf)
            return
        C.route_fc2(self.dH, self.w1_route, self.am2, M, B, self.dc2m, self.gb, self.dlogits, self.H,
                    self.params, self.m, self.v, self.gdump, self.off, self.adam_t, t_off, *a, True, self.route_rm,
                    self.route_ws, self.route_ctr)
        C.fc1_wgrad_adam(self.dH, self.a1, M, self.params, self.m, self.v, self.gdump, self.w1bf, self.w1tbf, self.off, self.adam_t, t_off, *a)
        C.conv2_bwd(self.dc2m, self.p1s, self.am1, self.w2q, x, idx, self.wslab1, self.wslab2, B)
        C.conv_adam(self.wslab1, self.wslab2, self.gb, B, self.params, self.m, self.v, self.gdump, self.w2r, self.w2q, self.off, self.adam_t, t_off, *a)

    def train_step(self, x: torch.Tensor, y: torch.Tensor) -> float:
        """Convenience: one eager step on a uint8 batch ``x`` [B,1,28,28] with labels ``y``; returns the loss."""
        B = int(y.shape[0])
        self.stats.zero_()
        self.train_step_async(x.contiguous(), y.to(torch.int64).contiguous(), None, B, self.stats, 1)
        self.adam_t += 1
        return float(self.stats[0]) / B

    @torch.no_grad()
    def logits_reference(self, x: torch.Tensor) -> torch.Tensor:
        return self.arena.module(x.float() / 255.0)


class _EvalSnapshot:
    """The weights one kind of evaluation pass reads, copied out of the engine.

    An evaluation pass runs on the learner's evaluation stream NEXT TO the
    training that follows it (the test pass beside the round's epoch, the
    validation pass beside the next round's), so it must not read the arena
    the optimizer is rewriting.  The copy is taken on the learner's stream at
    the point the pass's semantics fix (after the epoch / the aggregation):
    the fp32 ranges the forward kernels read (conv1 weight + bias, conv2 bias,
    l1 bias, l2 weight + bias; a few tens of KB) and the bf16 shadows (conv2,
    FC1, FC2; 13 MB).  Before, the passes sat between two epochs on the
    device's critical path: 0.45 ms of a 7.9 ms round (profiles/r5_cnn_gaps.md).
    """

    READ = ("conv1.weight", "conv1.bias", "conv2.bias", "l1.bias", "l2.weight", "l2.bias")

    def __init__(self, eng: "FusedCNNEngine") -> None:
        self.params = torch.zeros_like(eng.params)
        self.w2r = torch.zeros_like(eng.w2r)
        self.w1bf = torch.zeros_like(eng.w1bf)
        self.w2bf = None if eng.w2bf is None else torch.zeros_like(eng.w2bf)
        ends = list(eng.off[1:]) + [eng.params.numel()]
        spans = sorted((eng.off[_NAMES.index(n)], ends[_NAMES.index(n)]) for n in self.READ)
        self.ranges: List[Tuple[int, int]] = []
        for a, b in spans:  # adjacent parameters: one copy
            if self.ranges and self.ranges[-1][1] == a:
                self.ranges[-1] = (self.ranges[-1][0], b)
            else:
                self.ranges.append((a, b))
        self.done: Optional[torch.cuda.Event] = None  # end of the last pass that read this copy

    def take(self, eng: "FusedCNNEngine") -> None:
        """Enqueue the copy on the current stream: ONE launch of the multi-region
        copy kernel (csrc/fused_ops.hip; one blit kernel per region was ~45 us
        for a snapshot on the learner's stream, profiles/r5_cnn_gaps.md)."""
        dst = [self.params[a:b] for a, b in self.ranges] + [self.w2r, self.w1bf]
        src = [eng.params[a:b] for a, b in self.ranges] + [eng.w2r, eng.w1bf]
        if self.w2bf is not None:
            dst.append(self.w2bf)
            src.append(eng.w2bf)
        ops.ext().fused.multi_copy(dst, src)


class _EvalForward:
    """Forward-only view of a :class:`FusedCNNEngine` at 128 samples per launch.

    Evaluation has no optimizer step between batches, so it runs the same
    forward kernels (reading a :class:`_EvalSnapshot` of the engine's fp32
    parameters and bf16 shadows) on 128-sample batches: a quarter of the
    launches per pass, and the FC1 GEMM -- bound by streaming its 12.8 MB
    weight -- costs little more per launch at 128 rows than at 32.
    Per-sample losses and predictions do not depend on how the set is batched.
    """

    MROWS = 128

    def __init__(self, eng: FusedCNNEngine) -> None:
        self.eng = eng
        M, dev, bf = self.MROWS, eng.device, torch.bfloat16
        z = lambda *s, dt=torch.float32: torch.zeros(*s, dtype=dt, device=dev)  # noqa: E731
        self.p1, self.am1 = z(M * 196 * 32, dt=bf), z(M * 196 * 32, dt=torch.uint8)
        self.a1, self.am2 = z(M * FEAT, dt=bf), z(M * FEAT, dt=torch.uint8)
        self.slabs1 = z(eng.S1 * M * HID)
        self.H, self.dH = z(M * HID, dt=bf), z(M * HID, dt=bf)
        self.dlogits = z(M * 10)
        self.snaps: Dict[str, _EvalSnapshot] = {}

    def snapshot(self, name: str) -> _EvalSnapshot:
        """The weight copy the ``name`` pass (its captured graph) reads."""
        if name not in self.snaps:
            self.snaps[name] = _EvalSnapshot(self.eng)
        return self.snaps[name]

    def forward(self, x: torch.Tensor, labels: torch.Tensor, idx: Optional[torch.Tensor], B: int, stats: torch.Tensor,
                snap: _EvalSnapshot) -> None:
        e, C, M = self.eng, self.eng.C, self.MROWS
        if _CONV12:
            C.conv12_fwd(x, idx, snap.params, e.off, snap.w2r, None, self.am1, None, self.a1, self.am2, B, M)
        else:
            C.conv1_fwd(x, idx, snap.params, e.off, self.p1, self.am1, None, B)
            C.conv2_fwd(self.p1, snap.w2r, snap.params, e.off, self.a1, self.am2, B, M)
        C.gemm_skinny(self.a1, snap.w1bf, self.slabs1, M, HID, FEAT, e.S1)
        C.head(self.slabs1, e.S1, M, snap.params, e.off, labels, idx, B, False, self.H, self.dH, self.dlogits, stats,
               snap.w2bf)


class _EpochGraph:
    """One captured HIP graph per (dataset, batch plan)."""

    def __init__(self, graph: Optional[torch.cuda.CUDAGraph], key: Tuple) -> None:
        self.graph = graph
        self.key = key


class FusedCNNLearner(TorchLearner):
    """NodeLearner running the MNIST CNN through the fused HIP engine.

    Parameters, wire encoding and device snapshots come from
    :class:`TorchLearner` (same arena layout); ``fit``/``evaluate`` replay HIP
    graphs of whole epochs / evaluation passes.
    """

    def __init__(self, model: Any, data: Any, self_addr: str, epochs: int, device: Optional[torch.device] = None, use_graphs: bool = True, **kw) -> None:
        super().__init__(model, data, self_addr, epochs, device=device, fused_optimizer=False)
        if self.device.type != "cuda":
            raise RuntimeError("FusedCNNLearner needs an AMD GPU")
        opt = model.configure_optimizers() if hasattr(model, "configure_optimizers") else None
        lr = float(opt.param_groups[0]["lr"]) if opt is not None else 1e-3
        betas = tuple(opt.param_groups[0].get("betas", (0.9, 0.999))) if opt is not None else (0.9, 0.999)
        eps = float(opt.param_groups[0].get("eps", 1e-8)) if opt is not None else 1e-8
        wd = float(opt.param_groups[0].get("weight_decay", 0.0)) if opt is not None else 0.0
        self.engine = FusedCNNEngine(model, self.device, lr=lr, betas=betas, eps=eps, weight_decay=wd, arena=self.arena)
        self.use_graphs = use_graphs
        self._graphs: Dict[str, _EpochGraph] = {}
        self._lock = make_rlock("FusedCNNLearner._lock")  # fit() -> _validate() re-enters
        # one capture per pass key: fit() and the evaluation thread may both
        # reach _ensure_graph for a pass that has no graph yet
        self._graph_build_lock = make_lock("FusedCNNLearner._graph_build_lock")
        self._stream = private_stream(self.device)
        self._dirty_shadows = False
        self._eval_fwd = _EvalForward(self.engine)
        # asynchronous passes: metrics are read back by a completion thread;
        # the evaluation passes (validation, test) run on their own stream, on
        # weight snapshots, next to the training that follows them
        self._completions = HostCompletions(self_addr)
        # evaluation passes fill the gaps of the latency-bound training kernels
        # beside them: lowest queue priority, so the epoch's kernels dispatch first
        # (P2PFL_EVAL_STREAM_LOW=0: default priority)
        self._eval_stream = private_stream(self.device, 1 if _EVAL_LOW else 0)
        # completion events of the last RUN_AHEAD fits: the host may enqueue
        # round r + 1 while round r still trains, so the device never idles
        # while the stage machine moves between rounds (with a one-fit bound the
        # device waited ~0.3 ms per round for the host to enqueue the next
        # epoch: profiles/r5_cnn_gaps.md), and stays at most RUN_AHEAD fits ahead
        self._fit_hist: "collections.deque[torch.cuda.Event]" = collections.deque(maxlen=RUN_AHEAD)
        self._last_epoch_end: Optional[torch.cuda.Event] = None

    # -- parameters: keep the bf16 shadows in sync -------------------------
    def set_parameters(self, params) -> None:
        if isinstance(params, FlatParams) and params.flat.data_ptr() == self.engine.params.data_ptr():
            self._arena_changed()
            return  # the arena itself: weights and bf16 shadows are already current
        super().set_parameters(params)

    def _set_parameters(self, params) -> None:
        """The copy into the arena and the bf16 shadow refresh, both on the learner's
        stream inside set_parameters' hand-off (fit() does not wait on the caller's
        stream, so nothing it reads may be left there)."""
        super()._set_parameters(params)
        self.engine.pack_shadows()

    # -- plans ----------------------------------------------------------------
    def _plan(self, n: int, B: int) -> List[Tuple[int, int]]:
        return [(s, min(B, n - s)) for s in range(0, n, B)]

    def _graph_key(self, name: str, loader, train: bool):
        n = len(loader.dataset)
        B = loader.batch_size if train else _EvalForward.MROWS
        return self._plan(n, B), (name, n, B, loader.x.data_ptr(), loader.y.data_ptr())

    def _ensure_graph(self, name: str, loader, train: bool) -> "_EpochGraph":
        """The captured pass for ``loader`` (capturing it on first use).  Called
        WITHOUT ``self._lock``: waiting for the exclusive device gate can take as
        long as another peer's warm-up.  Recording a capture executes nothing, so
        the state the graph mutates (weights, Adam moments, step counter) is left
        untouched -- nothing to save or restore (see ``_capture``)."""
        from p2pfl_amd.learning.step_graph import GATE

        plan, key = self._graph_key(name, loader, train)
        g = self._graphs.get(name)
        if g is not None and g.key == key:
            return g
        with self._graph_build_lock:
            g = self._graphs.get(name)
            if g is None or g.key != key:
                import gc

                with GATE.shared():  # outside the exclusive section, never during another thread's capture
                    gc.collect()
                with GATE.exclusive():  # no other learner's GPU work during the capture
                    g = self._capture(name, loader, plan, train, key)
                self._graphs[name] = g
        return g

    def _run(self, name: str, loader, train: bool, perm: Optional[torch.Tensor]) -> torch.Tensor:
        """Enqueue a pass over ``loader``; returns a [steps, 2] stats tensor (loss sum, correct)."""
        from p2pfl_amd.learning.step_graph import GATE

        plan, _ = self._graph_key(name, loader, train)
        g = self._ensure_graph(name, loader, train)
        with GATE.shared():
            if perm is not None:
                g.perm.copy_(perm, non_blocking=True)
            if g.graph is not None:
                g.graph.replay()  # zeroes its stats itself (first node)
            else:
                g.stats.zero_()
                self._enqueue(name, loader, plan, train, g.perm, g.stats)
        return g.stats

    def _enqueue(self, name, loader, plan, train, perm, stats) -> None:
        x = loader.x.reshape(-1, 784)
        y = loader.y
        snap = None if train else self._eval_fwd.snapshot(name)
        chain = train and _FWD_IN_ADAM and _MERGED_ADAM and self.engine.mrows <= 64
        if train:
            self.engine._par = 0  # the captured sequence of A1 parities starts here on every replay
        for j, (s, b) in enumerate(plan):
            idx = perm[s : s + b]
            st = stats[j] if train else stats[0]
            if train:
                nxt = None
                if chain and j + 1 < len(plan):
                    s2, b2 = plan[j + 1]
                    nxt = (perm[s2 : s2 + b2], b2)
                self.engine.train_step_async(x, y, idx, b, st, j + 1, nxt=nxt, fwd_done=chain and j > 0)
            else:
                self._eval_fwd.forward(x, y, idx, b, st, snap)

    def _capture(self, name, loader, plan, train, key) -> _EpochGraph:
        n = len(loader.dataset)
        if not train:
            self._eval_fwd.snapshot(name)  # its buffers exist before (outside) the capture
        eg = _EpochGraph(None, key)
        eg.perm = torch.arange(n, dtype=torch.int64, device=self.device)
        eg.stats = torch.zeros((len(plan) if train else 1, 4), dtype=torch.float32, device=self.device)
        if not self.use_graphs:
            return eg
        from p2pfl_amd.learning.step_graph import no_gc

        # capture on a side stream.  Recording executes nothing, so the state the
        # graph mutates (weights, Adam moments, step counter) is untouched -- no
        # save / restore, which could also overwrite a set_parameters copy that
        # landed meanwhile
        with _CAPTURE_LOCK:
            torch.cuda.synchronize(self.device)
            graph = torch.cuda.CUDAGraph()
            with no_gc(collect=False), torch.cuda.graph(graph, stream=self._stream, capture_error_mode="relaxed"):
                eg.stats.zero_()  # in the graph: one launch fewer between two epochs
                self._enqueue(name, loader, plan, train, eg.perm, eg.stats)
            torch.cuda.synchronize(self.device)
        eg.graph = graph
        return eg

    # -- NodeLearner ------------------------------------------------------
    @staticmethod
    def _readback(stats: torch.Tensor) -> torch.Tensor:
        """Pinned host copy of a device stats tensor, enqueued behind the pass (under the
        shared device gate: the host allocator queries events, which must never happen
        beside another peer's capture -- hipErrorCapturedEvent)."""
        from p2pfl_amd.learning.step_graph import GATE

        with GATE.shared():
            host = torch.empty(stats.shape, dtype=stats.dtype, pin_memory=True)
            host.copy_(stats, non_blocking=True)
        return host

    def fit(self) -> None:
        if self.epochs <= 0 or self.model is None:
            return
        try:
            # the weights a fit reads arrive through set_parameters (its own hand-off);
            # the fit waits only for reads of the weights launched on other streams
            # since then (WeightGuard), so consecutive epochs pay no cross-queue wake-up
            with self._on_stream():
                self._fit_fused()
        finally:
            self._arena_changed()  # no snapshot taken mid-fit survives it

    def _fit_fused(self) -> None:
        """Enqueue the round's epochs (HIP-graph replays) and their validation passes.

        Returns as soon as the work is queued: per-step losses and validation
        metrics are logged by the completion thread when they land.  Everything
        that later reads or replaces the weights -- the gossip snapshot and
        its RCCL push, FedAvg, ``set_parameters`` -- is ordered behind the
        epoch by the stream.  The host runs at most ``RUN_AHEAD`` fits ahead of
        the GPU.
        """
        from p2pfl_amd.learning.step_graph import GATE

        self._interrupt.clear()
        self._arena_changed()
        if len(self._fit_hist) == RUN_AHEAD:
            self._fit_hist[0].synchronize()  # the fit RUN_AHEAD rounds back finished on the GPU
        self._ensure_graph("train", self.data.train_dataloader(), True)  # first-use captures outside the lock
        val = self.data.val_dataloader()
        if val is not None and len(val.dataset) > 0:
            self._ensure_graph("val", val, False)
        with self._lock:
            self.engine.reset_optimizer()  # Adam re-created per fit (reference quirk Q23)
            loader = self.data.train_dataloader()
            n, bs = len(loader.dataset), loader.batch_size
            steps = math.ceil(n / bs)
            cur = torch.cuda.current_stream(self.device)
            for epoch in range(self.epochs):
                if self._interrupt.is_set():
                    return
                if epoch:  # Adam step base for this epoch's graph (0 after the reset above)
                    self.engine.adam_t.fill_(epoch * steps)
                t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                t0.record(cur)
                with GATE.shared():  # pinned host buffer: never beside another peer's capture
                    perm = loader.permutation(host=True)
                stats = self._run("train", loader, True, perm)  # one H2D copy into the graph's buffer
                t1.record(cur)
                host = self._readback(stats)
                done = torch.cuda.Event()
                done.record(cur)
                base = self._step
                self._step += steps
                prev, self._last_epoch_end = self._last_epoch_end, t1
                self._completions.submit(done, lambda h=host, b=base, a=t0, z=t1, p=prev: self._log_epoch(h, b, steps, bs, n, a, z, p))
                self._validate_async()
            fit_done = torch.cuda.Event()
            fit_done.record(cur)
            self._fit_hist.append(fit_done)

    def _log_epoch(self, host: torch.Tensor, base: int, steps: int, bs: int, n: int, t0: Any, t1: Any, prev_end: Any = None) -> None:
        loss_sums = [row[0] for row in host.tolist()]
        every = max(1, self.log_every_n_steps)
        for j in range(steps):
            if (base + j + 1) % every == 0:
                self._log("train_loss", loss_sums[j] / min(bs, n - j * bs), step=base + j + 1)
        self.last_train_loss = sum(loss_sums) / n
        # GPU time of the replayed epoch (the host only enqueued it)
        ms = t0.elapsed_time(t1)
        logger.tracer.record(self._addr, "train_epoch_gpu", time.perf_counter() - ms * 1e-3, ms * 1e-3)
        if prev_end is not None:
            # device time from the previous epoch's end to this one's start: the
            # round's other GPU work (evaluation, readbacks, optimizer reset)
            # plus any idle time the host left between them
            gap = prev_end.elapsed_time(t0)
            logger.tracer.record(self._addr, "inter_epoch_gpu", time.perf_counter() - gap * 1e-3, gap * 1e-3)

    def _eval_async(self, name: str, loader, on_done) -> None:
        """Enqueue an evaluation pass of the weights as the current stream has
        them now; ``on_done(loss, metric)`` runs on the completion thread.

        The weights are copied on the current stream (the only cost left on its
        timeline); the pass itself runs on the evaluation stream beside whatever
        the current stream does next.  The evaluation passes share their
        activation buffers, so they stay serialised on that one stream."""
        self._ensure_graph(name, loader, False)  # first-use capture outside the lock
        snap = self._eval_fwd.snapshot(name)
        cur = torch.cuda.current_stream(self.device)
        side = self._stream_for_block() is not None if _EVAL_SIDE == "auto" else _EVAL_SIDE != "0"
        es = self._eval_stream if side else cur
        with self._lock:
            if snap.done is not None:
                cur.wait_event(snap.done)  # the previous pass on this copy finished reading it
            snap.take(self.engine)
            es.wait_stream(cur)
            with torch.cuda.stream(es):
                stats = self._run(name, loader, False, None)
                host = self._readback(stats[0, :2])
                ev = torch.cuda.Event()
                ev.record(es)
            snap.done = ev
        n = max(1, len(loader.dataset))

        def fin() -> None:
            loss, correct = host.tolist()
            on_done(loss / n, correct / n)

        self._completions.submit(ev, fin)
        return ev

    def _validate_async(self) -> None:
        loader = self.data.val_dataloader()
        if loader is None or len(loader.dataset) == 0:
            return
        step = self._step
        self._eval_async("val", loader, lambda loss, acc: (self._log("val_loss", loss, step=step), self._log("val_metric", acc, step=step)))

    def _validate(self) -> None:
        self._validate_async()
        self._completions.drain()

    def evaluate_async(self, on_results: Optional[Any] = None) -> bool:
        """Enqueue the test pass; results are logged (and handed to
        ``on_results``) when they land.  False when there is nothing to
        evaluate (``epochs == 0``, reference quirk Q18)."""
        if self.epochs <= 0 or self.model is None:
            return False

        def done(loss: float, acc: float) -> None:
            results = {"test_loss": loss, "test_metric": acc}
            for k, v in results.items():
                self._log(k, v)
            if on_results is not None:
                on_results(results)

        # the weights come from fit() / set_parameters on this learner's stream: no wait
        # on the caller's stream (a cross-queue wake-up ahead of the next epoch)
        with logger.span(self._addr, "evaluate"), self._on_stream(writes=False):
            self._eval_async("test", self.data.test_dataloader(), done)
        return True

    def evaluate(self) -> Dict[str, float]:
        box: Dict[str, float] = {}
        if not self.evaluate_async(box.update):
            return {}
        self._completions.drain()
        return box

    def drain(self, timeout: Optional[float] = None) -> bool:
        """Wait for every enqueued pass's host work (metrics) to finish."""
        return self._completions.drain(timeout)


def auto_learner(model: Any, data: Any, self_addr: str, epochs: int, **kw):
    """Pick the fastest learner for ``model`` on this machine."""
    from p2pfl_amd.models.cnn import CNN

    if isinstance(model, CNN) and torch.cuda.is_available() and ops.available():
        return FusedCNNLearner(model, data, self_addr, epochs, **kw)
    return TorchLearner(model, data, self_addr, epochs, **kw)
