"""Transports and the gossip / heartbeat machinery.

Transports: ``InMemoryCommunicationProtocol`` (in-process, device payloads),
``GrpcCommunicationProtocol`` (TCP / unix sockets).  The multi-process RCCL data
plane for one-peer-per-GPU deployments lives in :mod:`p2pfl_amd.parallel`.
"""

from p2pfl_amd.communication.protocol import BaseCommunicationProtocol, CommunicationProtocol

__all__ = ["CommunicationProtocol", "BaseCommunicationProtocol"]
