"""Transport-independent server logic.

Both the in-memory and the gRPC server delegate here so the delivery semantics
are written once (reference duplicates them in ``grpc_server.py:130-197`` and
``memory_server.py:123-186``):

* ``handle_message``: drop duplicates by hash, relay through the gossiper while
  ``ttl > 1`` (to direct neighbours except the source), execute the command;
  unknown commands and handler exceptions produce an error reply (which makes
  the sender drop the link, quirk Q13).
* ``handle_weights``: no dedupe, no relay; execute the command with
  ``weights/contributors/weight`` keyword arguments.
* ``handle_handshake`` / ``handle_disconnect``: add / remove the caller as a
  direct neighbour.
"""

from __future__ import annotations

import dataclasses
from typing import Any, Dict, List, Optional, Union

from p2pfl_amd.commands.command import Command
from p2pfl_amd.communication.messages import Message, WeightsMessage
from p2pfl_amd.management.logger import logger


class ServerCore:
    def __init__(self, addr: str, gossiper: Any, neighbors: Any, commands: Optional[List[Command]] = None) -> None:
        self.addr = addr
        self._gossiper = gossiper
        self._neighbors = neighbors
        self._commands: Dict[str, Command] = {}
        if commands:
            self.add_command(commands)

    def add_command(self, cmds: Union[Command, List[Command]]) -> None:
        if isinstance(cmds, Command):
            cmds = [cmds]
        for c in cmds:
            if not isinstance(c, Command):
                raise Exception("Command not valid")
            self._commands[c.get_name()] = c

    @property
    def commands(self) -> Dict[str, Command]:
        return self._commands

    # ------------------------------------------------------------------
    def handle_handshake(self, caller: str) -> Optional[str]:
        if self._neighbors.add(caller, non_direct=False, handshake_msg=False):
            return None
        return "Cannot add the node (duplicated or wrong direction)"

    def handle_disconnect(self, caller: str) -> None:
        self._neighbors.remove(caller, disconnect_msg=False)

    def handle_message(self, msg: Message) -> Optional[str]:
        if not self._gossiper.check_and_set_processed(msg.hash):
            return None
        logger.debug(self.addr, f"Received message from {msg.source} > {msg.cmd} {msg.args}")
        if msg.ttl > 1:
            relay = dataclasses.replace(msg, ttl=msg.ttl - 1, args=list(msg.args))
            pending = [n for n in self._neighbors.get_all(only_direct=True) if n != msg.source]
            self._gossiper.add_message(relay, pending)
        cmd = self._commands.get(msg.cmd)
        if cmd is None:
            logger.error(self.addr, f"Unknown command: {msg.cmd} from {msg.source}")
            return f"Unknown command: {msg.cmd}"
        try:
            cmd.execute(msg.source, msg.round, *msg.args)
        except Exception as e:
            err = f"Error while processing command: {msg.cmd} {msg.args}: {e}"
            logger.error(self.addr, err)
            return err
        return None

    def handle_weights(self, msg: WeightsMessage) -> Optional[str]:
        cmd = self._commands.get(msg.cmd)
        if cmd is None:
            logger.error(self.addr, f"Unknown command: {msg.cmd} from {msg.source}")
            return f"Unknown command: {msg.cmd}"
        logger.tracer.count(self.addr, "weights_bytes_recv", msg.nbytes())
        try:
            with logger.span(self.addr, "handle_weights", cmd=msg.cmd, src=msg.source):
                cmd.execute(
                    msg.source,
                    msg.round,
                    weights=msg.weights,
                    contributors=list(msg.contributors),
                    weight=msg.weight,
                )
        except Exception as e:
            err = f"Error while processing model: {msg.cmd}: {e}"
            logger.error(self.addr, err)
            return err
        return None
