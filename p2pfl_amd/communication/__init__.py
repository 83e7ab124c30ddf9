"""Transports and the gossip / heartbeat machinery.

Transports: ``InMemoryCommunicationProtocol`` (in-process, device payloads),
``GrpcCommunicationProtocol`` (TCP / unix sockets) and, for one peer per GPU,
``XgmiCommunicationProtocol`` (:mod:`p2pfl_amd.communication.xgmi`: node-local
control bus + RCCL point-to-point data plane over xGMI).
"""

from p2pfl_amd.communication.protocol import BaseCommunicationProtocol, CommunicationProtocol

__all__ = ["CommunicationProtocol", "BaseCommunicationProtocol"]
