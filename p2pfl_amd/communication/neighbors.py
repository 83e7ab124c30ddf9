"""Neighbour table (reference ``communication/neighbors.py:27-170``).

``addr -> NeighborEntry(conn, handle, last_beat)``.  A neighbour is *direct*
when it has a handle (gRPC stub, in-memory server object, ...) and
*non-direct* (known only through flooded heartbeats) otherwise.  Transports
subclass and implement ``connect``/``disconnect``.

Unlike the reference, transport calls (handshake / disconnect RPCs) never run
while the table lock is held, so a synchronous in-process transport cannot
deadlock two nodes that connect to each other at the same time.
"""

from __future__ import annotations

import threading
import time
from typing import Any, Dict, NamedTuple, Optional

from p2pfl_amd.management.logger import logger
from p2pfl_amd.utils.lockcheck import make_rlock


class NeighborEntry(NamedTuple):
    conn: Any
    handle: Any
    last_beat: float


class Neighbors:
    def __init__(self, self_addr: str) -> None:
        self.self_addr = self_addr
        self.neis: Dict[str, NeighborEntry] = {}
        self.neis_lock = make_rlock("Neighbors.neis_lock")
        self._on_change: list = []

    # -- transport hooks -------------------------------------------------
    def connect(self, addr: str, non_direct: bool = False, handshake_msg: bool = True) -> NeighborEntry:
        raise NotImplementedError

    def disconnect(self, addr: str, disconnect_msg: bool = True) -> None:
        raise NotImplementedError

    # -- change listeners (used to wake event-driven loops) --------------
    def add_listener(self, fn) -> None:
        self._on_change.append(fn)

    def _changed(self) -> None:
        for fn in list(self._on_change):
            try:
                fn()
            except Exception:
                pass

    # -- table operations ------------------------------------------------
    def refresh_or_add(self, addr: str, t: float) -> None:
        with self.neis_lock:
            e = self.neis.get(addr)
            if e is not None:
                self.neis[addr] = NeighborEntry(e.conn, e.handle, t)
                return
        self.add(addr, non_direct=True)

    def add(self, addr: str, non_direct: bool = False, handshake_msg: bool = True) -> bool:
        if addr == self.self_addr:
            logger.info(self.self_addr, "Cannot add itself")
            return False
        with self.neis_lock:
            if addr in self.neis and not (self.neis[addr].handle is None and not non_direct):
                logger.debug(self.self_addr, f"Cannot add duplicates. {addr} already exists.")
                return False
        try:
            entry = self.connect(addr, non_direct=non_direct, handshake_msg=handshake_msg)
        except Exception as e:
            logger.info(self.self_addr, f"Cannot add {addr}: {e}")
            return False
        with self.neis_lock:
            old = self.neis.get(addr)
            if old is not None and old.handle is not None:
                # raced with another add of the same direct neighbour
                self._close_entry(entry)
                return False
            self.neis[addr] = entry
        logger.info(self.self_addr, f"{'Discovered' if non_direct else 'Connected to'} {addr}")
        self._changed()
        return True

    def _close_entry(self, entry: NeighborEntry) -> None:
        pass

    def remove(self, addr: str, disconnect_msg: bool = True) -> None:
        with self.neis_lock:
            present = addr in self.neis
        if not present:
            return
        try:
            self.disconnect(addr, disconnect_msg=disconnect_msg)
        except Exception:
            pass
        with self.neis_lock:
            entry = self.neis.pop(addr, None)
        if entry is not None:
            self._close_entry(entry)
            logger.info(self.self_addr, f"Removed neighbor {addr}")
            self._changed()

    def get(self, addr: str) -> NeighborEntry:
        with self.neis_lock:
            return self.neis[addr]

    def get_all(self, only_direct: bool = False) -> Dict[str, NeighborEntry]:
        with self.neis_lock:
            neis = dict(self.neis)
        if only_direct:
            return {k: v for k, v in neis.items() if v.handle is not None}
        return neis

    def exists(self, addr: str) -> bool:
        with self.neis_lock:
            return addr in self.neis

    def clear_neighbors(self) -> None:
        for addr in list(self.get_all().keys()):
            self.remove(addr)

    @staticmethod
    def now() -> float:
        return time.time()
