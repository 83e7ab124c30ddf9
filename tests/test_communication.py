"""Transport / topology / fault tests (reference ``test/communication_test.py``), on both transports."""

from __future__ import annotations

import time

import pytest

from p2pfl_amd.node import Node
from p2pfl_amd.settings import Settings
from p2pfl_amd.utils import full_connection, wait_convergence


def _nodes(protocol, n):
    nodes = [Node(None, None, protocol=protocol) for _ in range(n)]
    for nd in nodes:
        nd.start()
    return nodes


@pytest.fixture
def two_nodes(protocol):
    nodes = _nodes(protocol, 2)
    yield nodes
    for nd in nodes:
        nd.stop()


@pytest.fixture
def four_nodes(protocol):
    nodes = _nodes(protocol, 4)
    yield nodes
    for nd in nodes:
        nd.stop()


def test_connect_invalid_node(protocol):
    n = Node(None, None, protocol=protocol)
    n.start()
    assert n.connect("google.es:80") is False
    assert n.connect("holadani.holaenrique") is False
    assert len(n.get_neighbors()) == 0
    n.stop()


def test_basic_node_pairing(two_nodes):
    n1, n2 = two_nodes
    assert n1.connect(n2.addr)
    wait_convergence(two_nodes, 1, only_direct=True)
    assert len(n1.get_neighbors(only_direct=True)) == len(n2.get_neighbors(only_direct=True)) == 1
    n2.disconnect(n1.addr)
    deadline = time.time() + Settings.HEARTBEAT_PERIOD * 2 + 1
    while time.time() < deadline and (n1.get_neighbors(only_direct=True) or n2.get_neighbors(only_direct=True)):
        time.sleep(0.05)
    assert len(n1.get_neighbors(only_direct=True)) == len(n2.get_neighbors(only_direct=True)) == 0


def test_full_connected(four_nodes):
    n1, n2, n3, n4 = four_nodes
    n1.connect(n2.addr)
    wait_convergence([n1, n2], 1, only_direct=True)
    full_connection(n3, [n1, n2])
    wait_convergence([n1, n2, n3], 2, only_direct=True)
    full_connection(n4, [n1, n2, n3])
    wait_convergence(four_nodes, 3, only_direct=True)
    n1.stop()
    wait_convergence([n2, n3, n4], 2, only_direct=True)
    n2.stop()
    wait_convergence([n3, n4], 1, only_direct=True)
    n3.stop()
    wait_convergence([n4], 0, only_direct=True)


def test_network_neighbors(four_nodes):
    """Star topology: non-direct neighbours are discovered through flooded heartbeats."""
    n1, n2, n3, n4 = four_nodes
    n1.connect(n2.addr)
    wait_convergence([n1, n2], 1, only_direct=False)
    n3.connect(n1.addr)
    wait_convergence([n1, n2, n3], 2, only_direct=False)
    n4.connect(n1.addr)
    wait_convergence(four_nodes, 3, only_direct=False)
    assert len(n2.get_neighbors(only_direct=True)) == 1
    n4.stop()
    wait_convergence([n1, n2, n3], 2, only_direct=False, wait=10)
    n3.stop()
    wait_convergence([n1, n2], 1, only_direct=False, wait=10)
    n2.stop()
    wait_convergence([n1], 0, only_direct=False, wait=10)


def test_bad_msg(two_nodes):
    """An unknown command gets an error reply and both sides drop the link."""
    n1, n2 = two_nodes
    n1.connect(n2.addr)
    wait_convergence(two_nodes, 1, only_direct=True)
    n1._communication_protocol.broadcast(n1._communication_protocol.build_msg("BAD_MSG"))
    deadline = time.time() + 2
    while time.time() < deadline and (n1.get_neighbors() or n2.get_neighbors()):
        time.sleep(0.05)
    assert len(n1.get_neighbors()) == len(n2.get_neighbors()) == 0


def test_node_abrupt_down(four_nodes):
    n1, n2, n3, n4 = four_nodes
    n1.connect(n2.addr)
    wait_convergence([n1, n2], 1, only_direct=True)
    full_connection(n3, [n1, n2])
    wait_convergence([n1, n2, n3], 2, only_direct=True)
    full_connection(n4, [n1, n2, n3])
    wait_convergence(four_nodes, 3, only_direct=True)
    # silent node: heartbeater stopped -> evicted by timeout
    n1._communication_protocol._heartbeater.stop()
    wait_convergence([n2, n3, n4], 2, only_direct=True, wait=10)
    n1.stop()
    # unreachable node: server stopped -> evicted on send failure
    n2._communication_protocol._server.stop()
    wait_convergence([n3, n4], 1, only_direct=True, wait=10)
    n2.stop()


def test_message_dedupe_and_relay(protocol):
    """Flooded messages reach non-direct nodes once (TTL relay + hash dedupe)."""
    from p2pfl_amd.commands.command import Command

    seen = []

    class Probe(Command):
        @staticmethod
        def get_name():
            return "probe"

        def execute(self, source, round, *args, **kwargs):
            seen.append((source, args))

    nodes = _nodes(protocol, 3)
    try:
        for nd in nodes:
            nd._communication_protocol.add_command(Probe())
        nodes[1].connect(nodes[0].addr)
        nodes[2].connect(nodes[1].addr)
        wait_convergence(nodes, 2, only_direct=False)
        proto = nodes[0]._communication_protocol
        proto.broadcast(proto.build_msg("probe", ["x"]))
        deadline = time.time() + 3
        while time.time() < deadline and len(seen) < 2:
            time.sleep(0.02)
        time.sleep(0.3)
        assert sorted(s for s, _ in seen) == [nodes[0].addr, nodes[0].addr]
        assert len(seen) == 2  # node1 and node2 each exactly once
    finally:
        for nd in nodes:
            nd.stop()


def test_grpc_address_parser():
    from p2pfl_amd.communication.grpc import AddressParser

    assert AddressParser("127.0.0.1:8080").get_parsed_address() == "127.0.0.1:8080"
    assert AddressParser("[::1]:8080").get_parsed_address() == "[::1]:8080"
    assert AddressParser("unix:///tmp/p.sock").get_parsed_address() == "unix:///tmp/p.sock"
    a = AddressParser("127.0.0.1").get_parsed_address()
    assert a.startswith("127.0.0.1:") and int(a.split(":")[1]) > 0
    with pytest.raises(ValueError):
        AddressParser("holadani.holaenrique").get_parsed_address()


def test_grpc_unix_socket(tmp_path):
    from p2pfl_amd.communication.grpc import GrpcCommunicationProtocol

    a = Node(None, None, address=f"unix://{tmp_path}/a.sock", protocol=GrpcCommunicationProtocol)
    b = Node(None, None, address=f"unix://{tmp_path}/b.sock", protocol=GrpcCommunicationProtocol)
    a.start()
    b.start()
    try:
        assert a.connect(b.addr)
        wait_convergence([a, b], 1, only_direct=True)
    finally:
        a.stop()
        b.stop()
