"""Federated round runner for one-peer-per-GPU jobs (``bench.py --aggregation allreduce``).

The default benchmark path is the full Node stage machine over the xGMI
transport; this runner is the comparison point without the protocol.

One round = the reference's per-round work for an all-train network
(``TrainStage`` -> ``GossipModelStage`` -> ``RoundFinishedStage``):

1. ``learner.evaluate()`` on the local test shard (metrics shared);
2. ``learner.fit()`` -- ``epochs`` passes over the local train shard plus the
   per-epoch validation pass;
3. FedAvg of the arenas of all peers (``CollectiveFedAvg`` over RCCL) and
   ``set_parameters`` of the result.

Gossip / training overlap: the last epoch's validation pass only reads the
trained weights, so the runner starts the weighted all-reduce of a snapshot
of them on RCCL's stream first and runs validation on the compute stream
meanwhile (``overlap_validation``); the aggregate is loaded once both are
done.  Same results as the serial order.

The control messages of the stage machine (votes, ``models_aggregated``,
``models_ready``) have no data-plane cost in this configuration and are
replaced by the collective's own synchronisation.
"""

from __future__ import annotations

import time
from dataclasses import dataclass, field
from typing import Dict, List

import torch

from p2pfl_amd.learning.arena import FlatParams
from p2pfl_amd.management.logger import logger
from p2pfl_amd.parallel.collective import CollectiveFedAvg


@dataclass
class RoundStats:
    seconds: float
    eval_s: float
    fit_s: float
    agg_s: float
    metrics: Dict[str, float] = field(default_factory=dict)


class FederatedRoundRunner:
    def __init__(self, learner, fedavg: CollectiveFedAvg, name: str = "peer", overlap_validation: bool = True) -> None:
        self.learner = learner
        self.overlap_validation = overlap_validation
        self.fedavg = fedavg
        self.name = name
        self.weight = float(learner.get_num_samples()[0])
        self.total_weight = fedavg.total_weight(self.weight)
        self.history: List[RoundStats] = []

    def _sync(self) -> None:
        if torch.cuda.is_available():
            torch.cuda.synchronize()

    def run_round(self, evaluate: bool = True) -> RoundStats:
        t0 = time.perf_counter()
        metrics = self.learner.evaluate() if evaluate else {}
        t1 = time.perf_counter()
        overlap = self.overlap_validation and hasattr(self.learner, "validate") and getattr(self.learner, "epochs", 0) > 0
        if overlap:
            self.learner.defer_final_validation = True
        try:
            with logger.span(self.name, "fit"):
                self.learner.fit()
        finally:
            if overlap:
                self.learner.defer_final_validation = False
        self._sync()
        t2 = time.perf_counter()
        with logger.span(self.name, "collective_fedavg"):
            params = self.learner.get_parameters()
            if overlap:
                # RCCL reduces a snapshot of the trained weights on its own
                # stream while the compute stream runs the validation pass
                pending = self.fedavg.aggregate_async(params.flat, self.weight, self.total_weight)
                self.learner.validate()
                agg = pending.wait()
                self.learner.set_parameters(params if agg is params.flat else FlatParams.from_flat(agg, params.layout))
            else:
                self.fedavg.aggregate_(params.flat, self.weight, self.total_weight)
                self.learner.set_parameters(params)
        self._sync()
        t3 = time.perf_counter()
        st = RoundStats(t3 - t0, t1 - t0, t2 - t1, t3 - t2, metrics)
        self.history.append(st)
        return st
