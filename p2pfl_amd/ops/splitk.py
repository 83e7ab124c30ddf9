"""Tile-arrival counters for split-K launches that reduce inside the kernel.

A split-K GEMM / convolution launch with counters (``csrc/gemm_core.h``)
needs one int per 128 x 128 output tile, zero when the launch starts; the
last K-slice to reach a tile reduces it and resets the counter, so the
array is zero again when the kernel ends.  Launches on one stream are
serialised, so a per-stream ring of counters is enough: each call takes the
next free slice, and calls captured into a HIP graph keep distinct slices
(the graph's capture stream has its own ring) -- two graphs replayed
concurrently on different streams never share a counter.
"""

from __future__ import annotations

import threading
from typing import Dict, List, Tuple

import torch

# Up to this many K-slices the last-arriving slice reduces a tile inside the
# launch (<= 256 KB of partials per tile); beyond it one wide slab reduction
# (csrc/conv.hip slab_sum) over the whole chip is faster than one workgroup
# reading every slice of its tile.
IN_LAUNCH_MAX_SPLITS = 4
RING = 1 << 18  # counters per stream (1 MiB)
_RINGS: Dict[Tuple[int, int], List] = {}
# virtual peers launch from several node threads: the ring cursor is shared
# per stream (torch hands out pooled streams), so taking a slice is atomic
_LOCK = threading.Lock()


# Counters of launches captured into a HIP graph belong to THAT graph: two
# graphs may be captured on the same pooled stream, and a per-stream ring that
# wraps around would hand a later capture (or eager launch) the slice an
# earlier graph baked in -- replayed concurrently on different streams, the
# two launches would corrupt each other's tile counts.  A capture therefore
# takes its slices from a ring of its own (kept alive by the graph object),
# which never wraps.
_SCOPE = threading.local()


class GraphCounters:
    """Counter ring owned by one captured graph (see :func:`graph_scope`)."""

    def __init__(self, device: torch.device, size: int = RING) -> None:
        self.buf = torch.zeros(size, dtype=torch.int32, device=device)
        self.used = 0

    def take(self, tiles: int) -> torch.Tensor:
        off = self.used
        if off + tiles > self.buf.numel():
            raise RuntimeError(f"graph counter ring exhausted ({off} + {tiles} > {self.buf.numel()})")
        self.used += (tiles + 15) // 16 * 16
        return self.buf[off : off + tiles]


class graph_scope:
    """``with graph_scope(ring): <capture>`` -- split-K launches captured by this
    thread take their counters from ``ring``."""

    def __init__(self, ring: GraphCounters) -> None:
        self.ring = ring

    def __enter__(self) -> GraphCounters:
        self.prev = getattr(_SCOPE, "ring", None)
        _SCOPE.ring = self.ring
        return self.ring

    def __exit__(self, *exc) -> None:
        _SCOPE.ring = self.prev


def counters(tiles: int, device: torch.device) -> torch.Tensor:
    """A zeroed int32 slice of ``tiles`` counters for one launch on the current stream."""
    if tiles > RING:
        raise ValueError(f"split-K launch with {tiles} tiles exceeds the counter ring")
    scoped = getattr(_SCOPE, "ring", None)
    if scoped is not None:
        return scoped.take(tiles)
    stream = torch.cuda.current_stream(device)
    key = (stream.device_index, stream.cuda_stream)
    with _LOCK:
        ring = _RINGS.get(key)
        if ring is None:
            ring = _RINGS[key] = [torch.zeros(RING, dtype=torch.int32, device=device), 0]
        if ring[1] + tiles > RING:
            ring[1] = 0
        off = ring[1]
        ring[1] += (tiles + 15) // 16 * 16
        return ring[0][off : off + tiles]


def tiles_of(rows: int, cols: int, tile: int = 128) -> int:
    return -(-rows // tile) * -(-cols // tile)


def slab_elems(rows: int, cols: int, variant: int = 0) -> int:
    """fp32 elements of one split-K slice: fragment-native tiles of the kernel the
    variant selects (128 x 128, or 256 x 256 with bit 6 or the ping-pong kernel's
    in-launch reduction; ``csrc/gemm_core.h`` SlabGeom), or the ping-pong kernel's
    row-major rows x cols of a separately reduced launch."""
    t = 256 if variant & (64 | 2048) else 128
    return max(rows * cols, -(-rows // t) * -(-cols // t) * t * t)
