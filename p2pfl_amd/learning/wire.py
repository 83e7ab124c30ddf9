"""Safe tensor wire codec.

The reference ships ``pickle.dumps([ndarray, ...])`` and unpickles whatever a
peer sends (``lightning_learner.py:113-138``) -- remote code execution for any
peer.  This codec carries only a JSON header and raw little-endian tensor
bytes, so decoding can never execute anything.

Layout::

    b"P2FA" | u32 version | u32 header_len | header (UTF-8 JSON) | pad to 64 B | payload

Header: ``{"kind": "flat", "layout": ParamLayout}`` for arena payloads (one
contiguous fp32 block -- one device-to-host copy to encode, one host-to-device
copy to decode), or ``{"kind": "dict", "tensors": [[name, dtype, shape,
offset, nbytes], ...]}`` for arbitrary tensor dicts.
"""

from __future__ import annotations

import json
import struct
from collections import OrderedDict
from typing import Mapping, Union

import numpy as np
import torch

from p2pfl_amd.learning.arena import FlatParams, ParamLayout
from p2pfl_amd.learning.exceptions import DecodingParamsError

MAGIC = b"P2FA"
VERSION = 1
_ALIGN = 64

_DTYPES = {
    "float32": torch.float32,
    "float64": torch.float64,
    "float16": torch.float16,
    "bfloat16": torch.bfloat16,
    "int64": torch.int64,
    "int32": torch.int32,
    "int16": torch.int16,
    "int8": torch.int8,
    "uint8": torch.uint8,
    "bool": torch.bool,
}


def _dtype_name(dt: torch.dtype) -> str:
    return str(dt).replace("torch.", "")


def _pack(header: dict, payload: bytes) -> bytes:
    h = json.dumps(header, separators=(",", ":")).encode()
    pre = MAGIC + struct.pack("<II", VERSION, len(h)) + h
    pad = (-len(pre)) % _ALIGN
    return pre + b"\0" * pad + payload


def _tensor_bytes(t: torch.Tensor) -> bytes:
    t = t.detach().contiguous().cpu()
    if t.dtype == torch.bfloat16:
        return t.view(torch.int16).numpy().tobytes()
    return t.numpy().tobytes()


def encode_params(params: Mapping[str, torch.Tensor]) -> bytes:
    if isinstance(params, FlatParams):
        return _pack({"kind": "flat", "layout": params.layout.to_json()}, _tensor_bytes(params.flat[: params.layout.numel]))
    entries, blobs, off = [], [], 0
    for name, t in params.items():
        b = _tensor_bytes(t)
        entries.append([name, _dtype_name(t.dtype), list(t.shape), off, len(b)])
        blobs.append(b)
        off += len(b)
    return _pack({"kind": "dict", "tensors": entries}, b"".join(blobs))


def decode_params(data: Union[bytes, bytearray, memoryview]) -> Union[FlatParams, "OrderedDict[str, torch.Tensor]"]:
    try:
        mv = memoryview(data)
        if bytes(mv[:4]) != MAGIC:
            raise DecodingParamsError("bad magic (not a p2pfl_amd tensor payload)")
        version, hlen = struct.unpack("<II", mv[4:12])
        if version != VERSION:
            raise DecodingParamsError(f"unsupported payload version {version}")
        header = json.loads(bytes(mv[12 : 12 + hlen]).decode())
        start = 12 + hlen
        start += (-start) % _ALIGN
        body = mv[start:]
        if header["kind"] == "flat":
            layout = ParamLayout.from_json(header["layout"])
            if len(body) != layout.numel * 4:
                raise DecodingParamsError("truncated flat payload")
            arr = np.frombuffer(body, dtype="<f4")
            flat = torch.from_numpy(arr.copy())
            return FlatParams.from_flat(flat, layout)
        if header["kind"] == "dict":
            out: "OrderedDict[str, torch.Tensor]" = OrderedDict()
            for name, dtype, shape, off, nbytes in header["tensors"]:
                dt = _DTYPES[dtype]
                raw = body[off : off + nbytes]
                if len(raw) != nbytes:
                    raise DecodingParamsError("truncated tensor payload")
                if dt == torch.bfloat16:
                    t = torch.from_numpy(np.frombuffer(raw, dtype="<i2").copy()).view(torch.bfloat16)
                else:
                    t = torch.from_numpy(np.frombuffer(raw, dtype=torch.empty(0, dtype=dt).numpy().dtype).copy())
                out[name] = t.reshape(shape)
            return out
        raise DecodingParamsError(f"unknown payload kind {header['kind']!r}")
    except DecodingParamsError:
        raise
    except Exception as e:
        raise DecodingParamsError(f"Error decoding parameters: {e}") from e
