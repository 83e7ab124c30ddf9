"""Collective FedAvg for one peer per GPU.

When every peer of a round is in the train set (the benchmark configuration,
``TRAIN_SET_SIZE >= peers``), the reference's gossip of disjoint partial
aggregates (``train_stage.py:114-177`` + ``aggregator.py:117-200``) converges to
exactly ``sum_i w_i * m_i / sum_i w_i`` on every peer.  Across GPUs of one node
that is a single weighted all-reduce: each peer scales its flat arena by
``w_i / W`` (one fused HIP kernel) and RCCL sums the arenas over xGMI.  Peers
outside the train set contribute weight 0 and receive the same result, which is
the reference's diffusion stage.

The flat fp32 arena is reduced in fixed-size buckets so the collective can be
overlapped with other work on a dedicated stream, and so RCCL's channels over
the 7 xGMI links stay saturated with large messages.
"""

from __future__ import annotations

import os
from dataclasses import dataclass
from typing import List, Optional

import torch
import torch.distributed as dist



@dataclass
class DistEnv:
    rank: int
    world_size: int
    local_rank: int
    device: torch.device

    @property
    def is_main(self) -> bool:
        return self.rank == 0


def init_distributed(backend: Optional[str] = None) -> DistEnv:
    """Initialise torch.distributed from torchrun env vars (single process if absent)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if torch.cuda.is_available():
        # one rank per GPU; more ranks than GPUs (tests on a 1-GPU box) share devices round-robin
        local_dev = local % torch.cuda.device_count()
        torch.cuda.set_device(local_dev)
        device = torch.device("cuda", local_dev)
    else:
        device = torch.device("cpu")
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # P2PFL_DIST_BACKEND=gloo: ranks sharing one GPU (RCCL rejects duplicate devices)
        backend = backend or os.environ.get("P2PFL_DIST_BACKEND") or ("nccl" if device.type == "cuda" else "gloo")
        kwargs = {"device_id": device} if backend == "nccl" else {}
        dist.init_process_group(backend=backend, rank=rank, world_size=world, **kwargs)
    return DistEnv(rank, world, local, device)


class CollectiveFedAvg:
    def __init__(self, env: DistEnv, bucket_bytes: int = 64 << 20) -> None:
        self.env = env
        self.bucket_elems = max(1, bucket_bytes // 4)

    def total_weight(self, weight: float) -> float:
        if self.env.world_size == 1:
            return float(weight)
        t = torch.tensor([float(weight)], dtype=torch.float64, device=self.env.device)
        dist.all_reduce(t)
        return float(t.item())

    def aggregate_(self, flat: torch.Tensor, weight: float, total: Optional[float] = None) -> torch.Tensor:
        """In place: ``flat <- sum_ranks (w_rank / W) * flat_rank``."""
        if self.env.world_size == 1:
            return flat
        if total is None:
            total = self.total_weight(weight)
        scale = float(weight) / total if total > 0 else 1.0 / self.env.world_size
        if scale != 1.0:
            flat.mul_(scale)
        for s in range(0, flat.numel(), self.bucket_elems):
            dist.all_reduce(flat[s : s + self.bucket_elems])
        return flat

    def aggregate_async(self, flat: torch.Tensor, weight: float, total: Optional[float] = None) -> "PendingFedAvg":
        """Start ``sum_ranks (w_rank / W) * flat_rank`` on a SNAPSHOT of ``flat``; returns a handle.

        The scaled snapshot is made by one kernel on the current (compute)
        stream; the bucketed all-reduces are issued with ``async_op=True`` so
        RCCL runs them on its own HIP stream, ordered after the snapshot but
        concurrent with whatever the compute stream does next (the round
        runner's validation pass).  ``flat`` itself stays untouched and
        readable meanwhile.  ``handle.wait()`` orders the current stream after
        the collective (no host block on RCCL) and returns the aggregate.
        """
        if self.env.world_size == 1:
            return PendingFedAvg(flat, [])
        if total is None:
            total = self.total_weight(weight)
        scale = float(weight) / total if total > 0 else 1.0 / self.env.world_size
        snap = flat * scale
        works = [dist.all_reduce(snap[s : s + self.bucket_elems], async_op=True) for s in range(0, snap.numel(), self.bucket_elems)]
        return PendingFedAvg(snap, works)

    def barrier(self) -> None:
        if self.env.world_size > 1:
            dist.barrier()

    def max_over_ranks(self, value: float) -> float:
        if self.env.world_size == 1:
            return value
        t = torch.tensor([value], dtype=torch.float64, device=self.env.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def gather_floats(self, value: float) -> List[float]:
        if self.env.world_size == 1:
            return [value]
        t = torch.tensor([value], dtype=torch.float64, device=self.env.device)
        out = [torch.zeros_like(t) for _ in range(self.env.world_size)]
        dist.all_gather(out, t)
        return [float(x.item()) for x in out]


class PendingFedAvg:
    """An in-flight :meth:`CollectiveFedAvg.aggregate_async`."""

    def __init__(self, result: torch.Tensor, works: list) -> None:
        self.result = result
        self._works = works

    def wait(self) -> torch.Tensor:
        for w in self._works:
            w.wait()
        self._works = []
        return self.result
