"""One-process-per-GPU runtime over RCCL (torch.distributed backend "nccl" == RCCL on ROCm)."""

from p2pfl_amd.parallel.collective import CollectiveFedAvg, DistEnv, init_distributed

__all__ = ["CollectiveFedAvg", "DistEnv", "init_distributed"]
