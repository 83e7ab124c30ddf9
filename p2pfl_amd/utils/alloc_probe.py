"""Caching-allocator probes for HIP-graph memory bugs.

A captured step graph replays fixed device addresses.  If anything it touches
lives outside the graph's private pool (a block PyTorch considers free, or
memory a library manages behind PyTorch's back), the graph keeps working only
as long as the allocator happens to hand the same blocks out again.
:func:`poison_free_blocks` takes every free cached block away (optionally
filling it with NaN), so the next replay runs against an allocator that must
map new segments -- the situation a profiler's own allocations create, which
is how the round-2 "NaN under rocprofv3" showed up
(``profiles/r3_nan_root_cause.md``; ``scripts/graph_poison.py``).
"""

from __future__ import annotations

import torch


def poison_free_blocks(dev: torch.device, fill: bool = True) -> list:
    """Allocate (and, with ``fill``, NaN-fill) every free block of the caching allocator."""
    keep = []
    sizes = [1 << s for s in range(30, 9, -1)]
    for sz in sizes:
        while True:
            free_cached = torch.cuda.memory_reserved(dev) - torch.cuda.memory_allocated(dev)
            if free_cached < sz:
                break
            before = torch.cuda.memory_reserved(dev)
            t = torch.empty(sz // 4, dtype=torch.float32, device=dev)
            if torch.cuda.memory_reserved(dev) > before:  # new segment: not a freed block
                del t
                break
            if fill:
                t.fill_(float("nan"))
            keep.append(t)
    torch.cuda.synchronize(dev)
    return keep
