"""Multi-process transport: gRPC control plane + torch.distributed weights data plane.

One process per GPU; weights move GPU-to-GPU with RCCL point-to-point over
xGMI (gloo on CPU).  See :mod:`p2pfl_amd.communication.dist.dist_protocol`.
"""

from p2pfl_amd.communication.dist.dist_protocol import DistCommunicationProtocol, DistDataPlane

__all__ = ["DistCommunicationProtocol", "DistDataPlane"]
