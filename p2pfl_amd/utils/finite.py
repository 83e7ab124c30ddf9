"""Debug-mode finiteness checks (``P2PFL_CHECK_FINITE=1``).

Localises the FIRST tensor of a run that goes non-finite: every model a node
receives, every FedAvg result, every ``set_parameters`` and every trained
epoch is checked (one device reduction + host sync each, so only in debug
runs).  The failure names the node, the stage and the round, which tells a
training divergence (finite in, non-finite after ``fit``) from a transport or
ordering bug (a received or aggregated arena non-finite while every input was
finite).
"""

from __future__ import annotations

import os
from typing import Any

import torch

from p2pfl_amd.management.logger import logger

ENABLED = os.environ.get("P2PFL_CHECK_FINITE") == "1"
# first failure of the process (node, message), for drivers that stop early
FIRST_FAILURE: "list" = []


class NonFiniteError(FloatingPointError):
    pass


def _flat(t: Any) -> torch.Tensor:
    return t.flat if hasattr(t, "flat") else t


def check(node: str, what: str, t: Any, **ctx: Any) -> None:
    """Raise :class:`NonFiniteError` if ``t`` (tensor or flat arena) holds a NaN/Inf."""
    if not ENABLED or t is None:
        return
    flat = _flat(t)
    if not isinstance(flat, torch.Tensor) or not flat.is_floating_point():
        return
    bad = int((~torch.isfinite(flat)).sum())
    if bad:
        msg = f"non-finite {what}: {bad} of {flat.numel()} elements" + "".join(f", {k}={v}" for k, v in ctx.items())
        logger.error(node, msg)
        if not FIRST_FAILURE:
            FIRST_FAILURE.append((node, msg))
        raise NonFiniteError(f"{node}: {msg}")
