"""Address parsing (reference ``grpc/address.py:26-99``).

Accepts ``host:port``, ``[v6]:port``, a bare host (a free port is picked) and
``unix:///absolute/path``.  ``get_parsed_address`` returns the canonical form
used as the node's identity.
"""

from __future__ import annotations

import os
import socket
from ipaddress import ip_address
from typing import Optional


class AddressParser:
    def __init__(self, address: str) -> None:
        self.host: Optional[str] = None
        self.port: Optional[int] = None
        self.is_v6: Optional[bool] = None
        self.unix_domain = False
        self._parse(address)

    @staticmethod
    def _free_port(v6: bool = False) -> int:
        fam = socket.AF_INET6 if v6 else socket.AF_INET
        with socket.socket(fam, socket.SOCK_STREAM) as s:
            s.bind(("", 0))
            return s.getsockname()[1]

    def _parse(self, address: str) -> None:
        if address.startswith("unix://"):
            if os.path.isabs(address[len("unix://") :]):
                self.unix_domain = True
                self.host = address
            return
        try:
            head, sep, tail = address.rpartition(":")
            if sep and head and not (head.count(":") and not head.startswith("[")):
                host, port = head, int(tail)
                if not 1 <= port <= 65535:
                    raise ValueError("Port number is invalid.")
            else:
                host, port = address, None
            host = host.strip("[]")
            v6 = ip_address(host).version == 6
            self.host, self.is_v6 = host, v6
            self.port = port if port is not None else self._free_port(v6)
        except ValueError:
            self.host = self.port = self.is_v6 = None

    def get_parsed_address(self) -> str:
        if self.unix_domain:
            if self.host is None:
                raise ValueError("Unix domain address is invalid.")
            return self.host
        if self.host is None:
            raise ValueError("The address is invalid.")
        return f"[{self.host}]:{self.port}" if self.is_v6 else f"{self.host}:{self.port}"
