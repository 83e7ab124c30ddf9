"""Client side of a transport (reference ``communication/client.py:25-89``).

:class:`Client` is the abstract contract.  :class:`BaseClient` implements the
transport-independent behaviour shared by every transport:

* message construction (random 63-bit hash, ``Settings.TTL``, round ``-1`` when
  unset);
* send semantics: resolve the neighbour handle, optionally open a temporary
  connection to a non-direct peer, invoke the transport, and on ANY failure or
  error reply evict the neighbour (reference ``grpc_client.py:159-179``,
  quirk Q13 preserved);
* broadcast = sequential unicast to all direct neighbours.

Subclasses provide ``_deliver(handle, msg)`` and ``_temporary_handle(addr)``.
"""

from __future__ import annotations

from abc import ABC, abstractmethod
from typing import Any, List, Optional

from p2pfl_amd.communication.exceptions import NeighborNotConnectedError
from p2pfl_amd.communication.messages import Message, WeightsMessage, new_message_hash
from p2pfl_amd.management.logger import logger
from p2pfl_amd.settings import Settings


class Client(ABC):
    @abstractmethod
    def build_message(self, cmd: str, args: Optional[List[str]] = None, round: Optional[int] = None) -> Any: ...

    @abstractmethod
    def build_weights(
        self,
        cmd: str,
        round: int,
        serialized_model: Any,
        contributors: Optional[List[str]] = None,
        weight: int = 1,
    ) -> Any: ...

    @abstractmethod
    def send(self, nei: str, msg: Any, create_connection: bool = False) -> None: ...

    @abstractmethod
    def broadcast(self, msg: Any, node_list: Optional[List[str]] = None) -> None: ...


class BaseClient(Client):
    def __init__(self, self_addr: str, neighbors: Any) -> None:
        self._self_addr = self_addr
        self._neighbors = neighbors

    # -- construction ----------------------------------------------------
    def build_message(self, cmd: str, args: Optional[List[str]] = None, round: Optional[int] = None) -> Message:
        return Message(
            source=self._self_addr,
            ttl=Settings.TTL,
            hash=new_message_hash(),
            cmd=cmd,
            args=[str(a) for a in (args or [])],
            round=-1 if round is None else int(round),
        )

    def build_weights(
        self,
        cmd: str,
        round: int,
        serialized_model: Any,
        contributors: Optional[List[str]] = None,
        weight: int = 1,
    ) -> WeightsMessage:
        return WeightsMessage(
            source=self._self_addr,
            round=int(round),
            weights=serialized_model,
            contributors=list(contributors or []),
            weight=int(weight),
            cmd=cmd,
        )

    # -- transport hooks -------------------------------------------------
    @abstractmethod
    def _deliver(self, handle: Any, msg: Any) -> Optional[str]:
        """Deliver ``msg`` through ``handle``; return an error string or None."""

    def _temporary_handle(self, addr: str) -> Any:
        """Handle for a one-off send to a non-direct peer (None if impossible)."""
        return None

    def _release_temporary(self, handle: Any) -> None:
        pass

    # -- send / broadcast ------------------------------------------------
    def send(self, nei: str, msg: Any, create_connection: bool = False) -> None:
        temp = None
        try:
            try:
                handle = self._neighbors.get(nei)[1]
            except KeyError as e:
                raise NeighborNotConnectedError(f"Neighbor {nei} not found.") from e
            if handle is None and create_connection:
                handle = temp = self._temporary_handle(nei)
            if handle is None:
                raise NeighborNotConnectedError(
                    "Neighbor not directly connected (no handle and create_connection is false)."
                )
            if isinstance(msg, WeightsMessage):
                logger.tracer.count(self._self_addr, "weights_bytes_sent", msg.nbytes())
                logger.tracer.count(self._self_addr, "weights_msgs_sent")
            error = self._deliver(handle, msg)
            if error:
                logger.error(self._self_addr, f"Error while sending a message: {msg.cmd}: {error}")
                self._neighbors.remove(nei, disconnect_msg=True)
        except Exception as e:
            logger.info(self._self_addr, f"Cannot send message {getattr(msg, 'cmd', '?')} to {nei}. Error: {e}")
            self._neighbors.remove(nei)
        finally:
            if temp is not None:
                self._release_temporary(temp)

    def broadcast(self, msg: Any, node_list: Optional[List[str]] = None) -> None:
        nodes = list(node_list) if node_list is not None else list(self._neighbors.get_all(only_direct=True).keys())
        for n in nodes:
            self.send(n, msg)
