"""Start one gRPC node and wait; run node2 against its port to start learning.

Reference: p2pfl/examples/node1.py.  ``python -m p2pfl_amd.examples.node1 6666``
"""

from __future__ import annotations

import argparse
import signal
import threading

from p2pfl_amd.data import MnistFederatedDM
from p2pfl_amd.models import MLP
from p2pfl_amd.node import Node


def main(argv=None) -> None:
    p = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    p.add_argument("port", type=int, help="port to listen on")
    p.add_argument("--timeout", type=float, default=None, help="stop after this many seconds (default: Ctrl-C)")
    args = p.parse_args(argv)
    node = Node(MLP(), MnistFederatedDM(sub_id=0, number_sub=2), address=f"127.0.0.1:{args.port}")
    node.start()
    print(f"node1 listening on {node.addr}; press Ctrl-C to stop", flush=True)
    done = threading.Event()
    signal.signal(signal.SIGINT, lambda *_: done.set())
    signal.signal(signal.SIGTERM, lambda *_: done.set())
    done.wait(args.timeout)
    node.stop()


if __name__ == "__main__":
    main()
