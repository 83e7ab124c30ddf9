"""Reference-compatible weight payloads, read without executing anything.

A stock p2pfl peer sends ``pickle.dumps([t.cpu().numpy() for t in
state_dict().values()])`` and loads whatever it receives with ``pickle.loads``
(reference ``lightning_learner.py:113-138``).  To federate with such peers
this module

* **reads** that payload with an allow-listed decoder: the opcode stream is
  checked first (``pickletools``; only the opcodes numpy's array pickling
  uses), then an ``Unpickler`` whose ``find_class`` resolves exactly the numpy
  array/dtype reconstructors (both the numpy<2 ``numpy.core`` and the numpy 2
  ``numpy._core`` spellings) and nothing else; the result must be a list of
  numeric ndarrays.  Any other global, opcode or object is rejected with
  :class:`DecodingParamsError` -- no peer can make this process run code;
* **writes** the same layout (``[ndarray, ...]`` in ``state_dict`` order)
  with numpy<2 module paths, which both numpy generations load.
"""

from __future__ import annotations

import io
import pickle
import pickletools
import struct
from typing import Any, List, Mapping

import numpy as np
import torch

from p2pfl_amd.learning.exceptions import DecodingParamsError

# (module, name) -> object; numpy 2 keeps numpy.core only as a deprecated alias
_ALLOWED = {
    ("numpy.core.multiarray", "_reconstruct"): ("numpy._core.multiarray", "_reconstruct"),
    ("numpy._core.multiarray", "_reconstruct"): ("numpy._core.multiarray", "_reconstruct"),
    ("numpy", "ndarray"): ("numpy", "ndarray"),
    ("numpy", "dtype"): ("numpy", "dtype"),
    ("numpy.core.numeric", "_frombuffer"): ("numpy._core.numeric", "_frombuffer"),
    ("numpy._core.numeric", "_frombuffer"): ("numpy._core.numeric", "_frombuffer"),
}

# every opcode numpy's ndarray / dtype pickling (protocols 2-5) can produce
_OPCODES = {
    "PROTO", "FRAME", "STOP", "MARK", "EMPTY_LIST", "APPEND", "APPENDS", "EMPTY_TUPLE", "TUPLE", "TUPLE1",
    "TUPLE2", "TUPLE3", "GLOBAL", "STACK_GLOBAL", "REDUCE", "BUILD", "MEMOIZE", "PUT", "BINPUT", "LONG_BINPUT",
    "GET", "BINGET", "LONG_BINGET", "BININT", "BININT1", "BININT2", "LONG1", "NONE", "NEWTRUE", "NEWFALSE",
    "SHORT_BINUNICODE", "BINUNICODE", "SHORT_BINBYTES", "BINBYTES", "BINBYTES8", "SHORT_BINSTRING", "BINSTRING",
    "BYTEARRAY8", "BINUNICODE8",
}

_NUMERIC_KINDS = set("biuf")  # bool, int, uint, float


def looks_like_pickle(data: Any) -> bool:
    try:
        mv = memoryview(data)
        return len(mv) >= 2 and mv[0] == 0x80 and 2 <= mv[1] <= 5
    except TypeError:
        return False


def _latin1_bytes(s: Any, encoding: str = "latin1") -> bytes:
    """Protocol-2 pickles spell ``bytes`` as ``_codecs.encode(str, 'latin1')``;
    only that exact form is accepted (no other codec can be reached)."""
    if not isinstance(s, str) or encoding != "latin1":
        raise DecodingParamsError("refusing _codecs.encode call in a weights payload")
    return s.encode("latin1")


def _empty_bytes(*args: Any) -> bytes:
    """Protocol 2 spells ``b""`` as ``bytes()``; nothing else is accepted."""
    if args:
        raise DecodingParamsError("refusing bytes(...) call in a weights payload")
    return b""


class _Restricted(pickle.Unpickler):
    def find_class(self, module: str, name: str) -> Any:
        if (module, name) == ("_codecs", "encode"):
            return _latin1_bytes
        if (module, name) in (("__builtin__", "bytes"), ("builtins", "bytes")):
            return _empty_bytes
        target = _ALLOWED.get((module, name))
        if target is None:
            raise DecodingParamsError(f"refusing global {module}.{name} in a weights payload")
        mod = __import__(target[0], fromlist=[target[1]])
        return getattr(mod, target[1])

    def persistent_load(self, pid: Any) -> Any:
        raise DecodingParamsError("persistent references are not allowed in a weights payload")


def decode_reference_payload(data: Any) -> List[torch.Tensor]:
    """The reference's pickled ``[ndarray, ...]`` as CPU tensors (nothing executed)."""
    raw = bytes(data)
    try:
        for op, _arg, _pos in pickletools.genops(raw):
            if op.name not in _OPCODES:
                raise DecodingParamsError(f"refusing pickle opcode {op.name} in a weights payload")
        obj = _Restricted(io.BytesIO(raw)).load()
    except DecodingParamsError:
        raise
    except Exception as e:
        raise DecodingParamsError(f"invalid reference weights payload: {e}") from e
    if not isinstance(obj, list):
        raise DecodingParamsError(f"reference payload must be a list of arrays, got {type(obj).__name__}")
    out = []
    for a in obj:
        if not isinstance(a, np.ndarray) or a.dtype.kind not in _NUMERIC_KINDS:
            raise DecodingParamsError("reference payload entries must be numeric numpy arrays")
        out.append(torch.from_numpy(np.array(a, copy=True, order="C")))  # (ascontiguousarray would make 0-d 1-d)
    return out


# ----------------------------------------------------------------------------
# emitter (hand-written opcode stream with numpy<2 paths)
# ----------------------------------------------------------------------------
def _uni(s: str) -> bytes:
    b = s.encode()
    return b"\x8c" + bytes([len(b)]) + b  # SHORT_BINUNICODE


def _int(v: int) -> bytes:
    if 0 <= v < 256:
        return b"K" + bytes([v])  # BININT1
    return b"J" + struct.pack("<i", v)  # BININT


def _bytes(b: bytes) -> bytes:
    if len(b) < 256:
        return b"C" + bytes([len(b)]) + b  # SHORT_BINBYTES
    if len(b) < (1 << 32):
        return b"B" + struct.pack("<I", len(b)) + b  # BINBYTES
    return b"\x8e" + struct.pack("<Q", len(b)) + b  # BINBYTES8


def _array(a: np.ndarray) -> bytes:
    a = np.array(a, copy=False, order="C") if a.flags.c_contiguous else np.array(a, order="C")
    dt = a.dtype.newbyteorder("<") if a.dtype.byteorder == ">" else a.dtype
    a = a.astype(dt, copy=False)
    code = dt.str[1:]  # e.g. 'f4', 'i8'
    order = "|" if dt.itemsize == 1 else "<"
    out = [b"cnumpy.core.multiarray\n_reconstruct\n", b"cnumpy\nndarray\n", _int(0), b"\x85", _bytes(b"b"), b"\x87R"]
    shape = b"(" + b"".join(_int(int(d)) for d in a.shape) + b"t" if a.ndim else b")"
    # dtype state: (3, byteorder, None, None, None, -1, -1, 0)
    dtype = (b"cnumpy\ndtype\n" + _uni(code) + b"\x89\x88\x87R" + b"(" + _int(3) + _uni(order) + b"NNN"
             + b"J\xff\xff\xff\xff" + b"J\xff\xff\xff\xff" + _int(0) + b"tb")
    out.append(b"(" + _int(1) + shape + dtype + b"\x89" + _bytes(a.tobytes()) + b"tb")
    return b"".join(out)


def encode_reference_payload(params: Mapping[str, torch.Tensor]) -> bytes:
    """``pickle.dumps([ndarray, ...])``-compatible bytes in ``state_dict`` order.

    Arena views go out in their original dtypes (the layout records them), so
    e.g. BatchNorm's int64 ``num_batches_tracked`` is an int64 array, as in the
    reference.
    """
    dtypes = None
    layout = getattr(params, "layout", None)
    if layout is not None:
        dtypes = list(layout.dtypes)
    body = [b"\x80\x03", b"]", b"("]  # PROTO 3, EMPTY_LIST, MARK
    for i, t in enumerate(params.values()):
        t = t.detach().cpu()
        if dtypes is not None and dtypes[i] != str(t.dtype).replace("torch.", ""):
            target = getattr(torch, dtypes[i])
            t = t.round().to(target) if not target.is_floating_point else t.to(target)
        if t.dtype == torch.bfloat16:
            t = t.float()
        body.append(_array(t.contiguous().numpy()))
    body.append(b"e.")  # APPENDS, STOP
    return b"".join(body)
