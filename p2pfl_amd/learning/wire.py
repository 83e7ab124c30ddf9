"""Safe tensor wire codec.

The reference ships ``pickle.dumps([ndarray, ...])`` and unpickles whatever a
peer sends (``lightning_learner.py:113-138``) -- remote code execution for any
peer.  This codec carries only a JSON header and raw little-endian tensor
bytes, so decoding can never execute anything.

Layout (v2)::

    b"P2FA" | u32 version | u32 header_len | u32 crc32c(payload) | u64 payload_len |
    header (UTF-8 JSON) | pad to 64 B | payload

The frame is validated by native code (``csrc/host/wire_frame.cpp``, loaded
with ctypes from ``p2pfl_amd/_p2fa.so``) before any byte of it is
interpreted: bounds of every length field and the CRC32C of the payload, so a
truncated or corrupted model is rejected instead of being averaged into the
federation.  That library is what the host sanitizer test fuzzes under
ASan/UBSan (``tests/test_native_sanitizers.py``).  Without the library the
same checks run in Python.  v1 frames (no checksum) are refused.

Interoperability with stock reference peers: :mod:`p2pfl_amd.learning.refpickle`
reads and writes the reference's ``pickle.dumps([ndarray, ...])`` payload with
an allow-listed, non-executing unpickler; :func:`decode_params` recognises it
by its pickle protocol header.

Header: ``{"kind": "flat", "layout": ParamLayout}`` for arena payloads (one
contiguous fp32 block -- one device-to-host copy to encode, one host-to-device
copy to decode), or ``{"kind": "dict", "tensors": [[name, dtype, shape,
offset, nbytes], ...]}`` for arbitrary tensor dicts.
"""

from __future__ import annotations

import ctypes
import json
import os
import struct
from collections import OrderedDict
from typing import Mapping, Union

import numpy as np
import torch

from p2pfl_amd.learning.arena import FlatParams, ParamLayout
from p2pfl_amd.learning.exceptions import DecodingParamsError

MAGIC = b"P2FA"
VERSION = 2
_ALIGN = 64
_PREFIX = 24  # magic, version, header_len, crc32c, payload_len


class _Frame(ctypes.Structure):
    _fields_ = [
        ("version", ctypes.c_uint32),
        ("header_off", ctypes.c_uint64),
        ("header_len", ctypes.c_uint64),
        ("payload_off", ctypes.c_uint64),
        ("payload_len", ctypes.c_uint64),
        ("crc", ctypes.c_uint32),
    ]


_ERRORS = {1: "truncated frame", 2: "bad magic (not a p2pfl_amd tensor payload)", 3: "unsupported payload version",
           4: "bad header length", 5: "truncated or oversized payload", 6: "payload checksum mismatch"}
_lib = None


def _addr(mv: memoryview):
    """(c_void_p, keepalive) for a contiguous byte view, without copying when possible."""
    if not mv.readonly:
        buf = (ctypes.c_char * len(mv)).from_buffer(mv)
        return ctypes.cast(buf, ctypes.c_void_p), buf
    obj = mv.obj
    if isinstance(obj, bytes) and len(obj) == len(mv):
        cp = ctypes.c_char_p(obj)  # points into the bytes object itself
        return ctypes.cast(cp, ctypes.c_void_p), cp
    data = mv.tobytes()
    cp = ctypes.c_char_p(data)
    return ctypes.cast(cp, ctypes.c_void_p), (cp, data)


def _native():
    """ctypes handle of the native frame library, or None."""
    global _lib
    if _lib is None:
        path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_p2fa.so")
        try:
            lib = ctypes.CDLL(path)
            lib.p2fa_crc32c.restype = ctypes.c_uint32
            lib.p2fa_crc32c.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32]
            lib.p2fa_validate.restype = ctypes.c_int
            lib.p2fa_validate.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(_Frame)]
            _lib = lib
        except OSError:
            _lib = False
    return _lib or None


def _crc_table():
    t = []
    for i in range(256):
        c = i
        for _ in range(8):
            c = (c >> 1) ^ 0x82F63B78 if c & 1 else c >> 1
        t.append(c)
    return t


_TABLE = None


def crc32c(data) -> int:
    """CRC32C of a bytes-like object (native when available)."""
    mv = memoryview(data).cast("B")
    lib = _native()
    if lib is not None:
        ptr, _keep = _addr(mv)
        return int(lib.p2fa_crc32c(ptr, len(mv), 0))
    global _TABLE
    if _TABLE is None:
        _TABLE = _crc_table()
    c = 0xFFFFFFFF
    for b in mv.tobytes():
        c = _TABLE[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def _validate(mv: memoryview):
    """(version, header bytes, payload memoryview) of a checked frame."""
    lib = _native()
    n = len(mv)
    if lib is not None:
        fr = _Frame()
        ptr, _keep = _addr(mv)
        rc = lib.p2fa_validate(ptr, n, ctypes.byref(fr))
        if rc != 0:
            raise DecodingParamsError(_ERRORS.get(rc, f"invalid frame ({rc})"))
        return (
            fr.version,
            bytes(mv[fr.header_off : fr.header_off + fr.header_len]),
            mv[fr.payload_off : fr.payload_off + fr.payload_len],
        )
    # pure-Python twin of p2fa_validate
    if n < 12:
        raise DecodingParamsError(_ERRORS[1])
    if bytes(mv[:4]) != MAGIC:
        raise DecodingParamsError(_ERRORS[2])
    version, hlen = struct.unpack("<II", mv[4:12])
    if version != 2:  # v1 (no checksum) is refused, like the native validator
        raise DecodingParamsError(_ERRORS[3])
    if n < _PREFIX:
        raise DecodingParamsError(_ERRORS[1])
    if hlen > n - _PREFIX:
        raise DecodingParamsError(_ERRORS[4])
    crc, plen = struct.unpack("<IQ", mv[12:24])
    start = -(-(_PREFIX + hlen) // _ALIGN) * _ALIGN
    if start > n or plen != n - start:
        raise DecodingParamsError(_ERRORS[5])
    body = mv[start:]
    if crc32c(body) != crc:
        raise DecodingParamsError(_ERRORS[6])
    return 2, bytes(mv[_PREFIX : _PREFIX + hlen]), body

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
    pre = MAGIC + struct.pack("<IIIQ", VERSION, len(h), crc32c(payload), len(payload)) + h
    pad = (-len(pre)) % _ALIGN
    return pre + b"\0" * pad + payload


def _tensor_bytes(t: torch.Tensor) -> bytes:
    t = t.detach().contiguous().cpu()
    if t.dtype == torch.bfloat16:
        return t.view(torch.int16).numpy().tobytes()
    return t.numpy().tobytes()


def encode_params(params: Mapping[str, torch.Tensor]) -> bytes:
    """This codec's frame; with ``Settings.WIRE_FORMAT == "reference"`` the
    reference's pickled array list instead (for federating with stock p2pfl peers)."""
    from p2pfl_amd.settings import Settings

    if Settings.WIRE_FORMAT == "reference":
        from p2pfl_amd.learning.refpickle import encode_reference_payload

        return encode_reference_payload(params)
    if isinstance(params, FlatParams):
        return _pack({"kind": "flat", "layout": params.layout.to_json()}, _tensor_bytes(params.flat[: params.layout.numel]))
    entries, blobs, off = [], [], 0
    for name, t in params.items():
        b = _tensor_bytes(t)
        entries.append([name, _dtype_name(t.dtype), list(t.shape), off, len(b)])
        blobs.append(b)
        off += len(b)
    return _pack({"kind": "dict", "tensors": entries}, b"".join(blobs))


def decode_params(data: Union[bytes, bytearray, memoryview]) -> Union[FlatParams, "OrderedDict[str, torch.Tensor]", list]:
    """Decode a payload: this codec's frame, or (a list of tensors) the
    reference's pickled ``[ndarray, ...]`` read by the allow-listed decoder."""
    from p2pfl_amd.learning import refpickle

    if refpickle.looks_like_pickle(data):
        return refpickle.decode_reference_payload(data)
    try:
        mv = memoryview(data).cast("B")
        _version, hbytes, body = _validate(mv)
        header = json.loads(hbytes.decode())
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
