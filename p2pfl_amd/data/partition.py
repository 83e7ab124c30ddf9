"""Federated partitioners.

* :func:`iid_shard`     -- contiguous shard ``sub_id`` of ``number_sub``
  (reference ``mnistfederated_dm.py:106-118``);
* :func:`label_sorted`  -- sort by label first, then shard: the reference's
  non-IID mode (``:87-90``), at most ~2 classes per node;
* :func:`dirichlet`     -- per-class Dirichlet(alpha) proportions over nodes
  (BASELINE config 3), deterministic in ``seed``.
"""

from __future__ import annotations

from typing import List

import numpy as np
import torch


def iid_shard(n: int, sub_id: int, number_sub: int) -> torch.Tensor:
    if sub_id + 1 > number_sub:
        raise ValueError(f"Not exist the subset {sub_id}")
    rows = n // number_sub
    return torch.arange(sub_id * rows, (sub_id + 1) * rows)


def label_sorted(labels: torch.Tensor, sub_id: int, number_sub: int) -> torch.Tensor:
    order = torch.sort(labels, stable=True).indices
    return order[iid_shard(len(labels), sub_id, number_sub)]


def dirichlet(labels: torch.Tensor, sub_id: int, number_sub: int, alpha: float = 0.5, seed: int = 0) -> torch.Tensor:
    if sub_id + 1 > number_sub:
        raise ValueError(f"Not exist the subset {sub_id}")
    rng = np.random.default_rng(seed)
    y = labels.numpy()
    parts: List[List[int]] = [[] for _ in range(number_sub)]
    for c in np.unique(y):
        idx = np.flatnonzero(y == c)
        rng.shuffle(idx)
        p = rng.dirichlet(np.full(number_sub, alpha))
        cuts = (np.cumsum(p) * len(idx)).astype(int)[:-1]
        for k, chunk in enumerate(np.split(idx, cuts)):
            parts[k].extend(chunk.tolist())
    mine = np.array(sorted(parts[sub_id]), dtype=np.int64)
    return torch.from_numpy(mine)
