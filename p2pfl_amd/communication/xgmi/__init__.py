"""xGMI transport: node-local control bus + RCCL point-to-point data plane."""

from p2pfl_amd.communication.xgmi.data_plane import SimFabric, XgmiDataPlane
from p2pfl_amd.communication.xgmi.xgmi_protocol import XgmiCommunicationProtocol, XgmiJob, XgmiSimNetwork

__all__ = ["XgmiCommunicationProtocol", "XgmiJob", "XgmiSimNetwork", "XgmiDataPlane", "SimFabric"]
