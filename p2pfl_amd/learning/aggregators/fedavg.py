"""Federated Averaging (McMahan et al. 2016) on flat arenas.

Reference: ``aggregators/fedavg.py:28-60`` loops ``accum[layer] += m[layer]*w``
over every model and layer (k x L torch ops, re-run for every gossip send).
Here every model is (or is converted to) a :class:`FlatParams` arena and the
whole average is ONE fused HIP kernel (``ops.weighted_average``): k input
pointers, fp32 accumulation, normalisation folded in, 16-byte vector loads,
grid sized for HBM3E bandwidth.  On CPU tensors the same math runs in torch.
"""

from __future__ import annotations

from typing import Any, Dict, List, Tuple

import torch

from p2pfl_amd import ops
from p2pfl_amd.learning.aggregators.aggregator import Aggregator, NoModelsToAggregateError
from p2pfl_amd.learning.arena import FlatParams, flatten


class FedAvg(Aggregator):
    """Sample-weighted mean of the models."""

    def aggregate(self, models: Dict[str, Tuple[Any, int]]) -> FlatParams:
        if len(models) == 0:
            raise NoModelsToAggregateError(f"({self.node_name}) Trying to aggregate models when there is no models")
        # fixed summation order (by contributor key), so every node that
        # aggregates the same models gets the bitwise-same result whatever
        # order they arrived in
        entries = [models[k] for k in sorted(models)]
        ref = entries[-1][0]
        device = next(iter(ref.values())).device if len(ref) else torch.device("cpu")
        flats: List[FlatParams] = [flatten(m, device=device) for m, _ in entries]
        layout = flats[0].layout
        for f in flats[1:]:
            if not f.layout.compatible(layout):
                raise ValueError("Cannot average models with different layouts")
        weights = [float(w) for _, w in entries]
        out = ops.weighted_average([f.flat for f in flats], weights)
        result = FlatParams.from_flat(out, layout)
        if not isinstance(ref, FlatParams):
            # preserve the caller's key order/names for plain dicts
            renamed = FlatParams()
            for (name, _), view in zip(ref.items(), result.values()):
                renamed[name] = view
            renamed.flat, renamed.layout = result.flat, result.layout
            return renamed
        return result
