"""gRPC transport (same service/messages as the reference ``node.proto``)."""

from p2pfl_amd.communication.grpc.address import AddressParser
from p2pfl_amd.communication.grpc.grpc_protocol import (
    GrpcClient,
    GrpcCommunicationProtocol,
    GrpcNeighbors,
    GrpcServer,
)

__all__ = ["AddressParser", "GrpcClient", "GrpcCommunicationProtocol", "GrpcNeighbors", "GrpcServer"]
