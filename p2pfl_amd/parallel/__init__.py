"""LEGACY comparison path: FedAvg as one weighted RCCL all-reduce (round 1).

Not the product.  The framework's federated round is the p2pfl protocol --
``Node`` + stages + gossip of partial aggregates over the xGMI transport
(:mod:`p2pfl_amd.communication.xgmi`) + the HIP FedAvg kernel.  This package
keeps the round-1 runner (one process per GPU, ``torch.distributed`` backend
"nccl" == RCCL, every round a weighted all-reduce of the arenas) only for
``bench.py --aggregation allreduce`` and ``--impl reference``, which measured
the reference-equivalent baseline quoted in ``BASELINE.md``.
"""

from p2pfl_amd.parallel.collective import CollectiveFedAvg, DistEnv, init_distributed

__all__ = ["CollectiveFedAvg", "DistEnv", "init_distributed"]
