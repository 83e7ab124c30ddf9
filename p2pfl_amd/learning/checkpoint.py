"""On-disk checkpoints of a peer's flat parameter arena.

The reference has no checkpointing (Lightning's is disabled,
``lightning_learner.py:188``); its only serialized model form is the gossip
wire layout (an ordered list of arrays mapped positionally onto the
receiver's keys).  Here a checkpoint is that same ordered layout made
explicit: one safetensors file holding the contiguous fp32 arena (plus any
optional extra tensors, e.g. Adam moments) and, in the safetensors metadata,
a JSON manifest -- parameter names, shapes, dtypes and arena offsets
(:class:`~p2pfl_amd.learning.arena.ParamLayout`) and free-form run metadata
(round, experiment, node address, samples).

Loading executes nothing from the file (safetensors + JSON only).  Writes
go to a temporary file that is atomically renamed, so a crash never leaves a
truncated checkpoint.
"""

from __future__ import annotations

import json
import os
import tempfile
from typing import Any, Dict, Mapping, Optional, Tuple

import torch
from safetensors import safe_open
from safetensors.torch import save_file

from p2pfl_amd.learning.arena import FlatParams, ParamLayout, flatten

FORMAT = "p2pfl_amd.checkpoint/1"


class CheckpointError(Exception):
    """The file is not a p2pfl_amd checkpoint or does not match the model."""


def save_checkpoint(
    path: str,
    params: Mapping[str, torch.Tensor],
    meta: Optional[Dict[str, Any]] = None,
    extra: Optional[Mapping[str, torch.Tensor]] = None,
) -> str:
    """Write ``params`` (a :class:`FlatParams` or any name->tensor mapping) to ``path``."""
    fp = params if isinstance(params, FlatParams) else flatten(params)
    from p2pfl_amd.learning.arena import reading

    with reading(fp):  # a learner's live weights: after its last write (WeightGuard)
        tensors = {"arena": fp.flat.detach().to("cpu", torch.float32).contiguous()}
    for k, v in (extra or {}).items():
        if k == "arena":
            raise ValueError("'arena' is reserved")
        tensors[k] = v.detach().to("cpu").contiguous()
    metadata = {
        "format": FORMAT,
        "layout": json.dumps(fp.layout.to_json()),
        "meta": json.dumps(meta or {}),
    }
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    fd, tmp = tempfile.mkstemp(prefix=".ckpt-", suffix=".tmp", dir=d)
    os.close(fd)
    try:
        save_file(tensors, tmp, metadata=metadata)
        os.replace(tmp, path)
    finally:
        if os.path.exists(tmp):
            os.unlink(tmp)
    return path


def load_checkpoint(
    path: str, device: Optional[torch.device] = None, expect: Optional[ParamLayout] = None
) -> Tuple[FlatParams, Dict[str, Any], Dict[str, torch.Tensor]]:
    """Read a checkpoint: (parameters as arena views, run metadata, extra tensors).

    ``expect``: a layout the parameters must match (shapes and order), e.g.
    the receiving learner's; a mismatch raises :class:`CheckpointError`.
    """
    try:
        with safe_open(path, framework="pt", device="cpu") as f:
            md = f.metadata() or {}
            if md.get("format") != FORMAT:
                raise CheckpointError(f"{path}: not a {FORMAT} file")
            layout = ParamLayout.from_json(json.loads(md["layout"]))
            meta = json.loads(md.get("meta", "{}"))
            flat = f.get_tensor("arena")
            extra = {k: f.get_tensor(k) for k in f.keys() if k != "arena"}
    except CheckpointError:
        raise
    except Exception as e:  # malformed header, missing keys, bad JSON
        raise CheckpointError(f"{path}: unreadable checkpoint ({e})") from e
    if flat.dim() != 1 or flat.numel() < layout.numel:
        raise CheckpointError(f"{path}: arena has {flat.numel()} elements, layout needs {layout.numel}")
    if expect is not None and tuple(expect.shapes) != tuple(layout.shapes):
        raise CheckpointError(f"{path}: parameter shapes do not match the model")
    if device is not None:
        flat = flat.to(device)
    return FlatParams.from_flat(flat, layout), meta, extra
