"""Runtime-built protobuf classes for ``node.proto``.

``protoc``/``grpcio-tools`` are not available in this image, so the file
descriptor is assembled programmatically with ``descriptor_pb2`` and the
message classes are obtained from the message factory.  The resulting wire
format is byte-identical to protoc-generated code for the same schema.
"""

from __future__ import annotations

from google.protobuf import descriptor_pb2, descriptor_pool, empty_pb2, message_factory

_F = descriptor_pb2.FieldDescriptorProto


def _add_field(msg, name: str, number: int, ftype: int, repeated: bool = False, optional: bool = False, oneof=None):
    f = msg.field.add()
    f.name = name
    f.json_name = name
    f.number = number
    f.type = ftype
    f.label = _F.LABEL_REPEATED if repeated else _F.LABEL_OPTIONAL
    if optional:
        f.proto3_optional = True
        f.oneof_index = oneof
    return f


def _build_file() -> descriptor_pb2.FileDescriptorProto:
    fd = descriptor_pb2.FileDescriptorProto()
    fd.name = "p2pfl_amd/node.proto"
    fd.package = "node"
    fd.syntax = "proto3"
    fd.dependency.append("google/protobuf/empty.proto")

    m = fd.message_type.add(name="Message")
    _add_field(m, "source", 1, _F.TYPE_STRING)
    _add_field(m, "ttl", 2, _F.TYPE_INT32)
    _add_field(m, "hash", 3, _F.TYPE_INT64)
    _add_field(m, "cmd", 4, _F.TYPE_STRING)
    _add_field(m, "args", 5, _F.TYPE_STRING, repeated=True)
    m.oneof_decl.add(name="_round")
    _add_field(m, "round", 6, _F.TYPE_INT32, optional=True, oneof=0)

    w = fd.message_type.add(name="Weights")
    _add_field(w, "source", 1, _F.TYPE_STRING)
    _add_field(w, "round", 2, _F.TYPE_INT32)
    _add_field(w, "weights", 3, _F.TYPE_BYTES)
    _add_field(w, "contributors", 4, _F.TYPE_STRING, repeated=True)
    _add_field(w, "weight", 5, _F.TYPE_INT32)
    _add_field(w, "cmd", 6, _F.TYPE_STRING)

    h = fd.message_type.add(name="HandShakeRequest")
    _add_field(h, "addr", 1, _F.TYPE_STRING)

    r = fd.message_type.add(name="ResponseMessage")
    r.oneof_decl.add(name="_error")
    _add_field(r, "error", 1, _F.TYPE_STRING, optional=True, oneof=0)

    svc = fd.service.add(name="NodeServices")
    for name, inp, out in (
        ("handshake", ".node.HandShakeRequest", ".node.ResponseMessage"),
        ("disconnect", ".node.HandShakeRequest", ".google.protobuf.Empty"),
        ("send_message", ".node.Message", ".node.ResponseMessage"),
        ("send_weights", ".node.Weights", ".node.ResponseMessage"),
    ):
        svc.method.add(name=name, input_type=inp, output_type=out)
    return fd


_pool = descriptor_pool.DescriptorPool()
_empty_fd = descriptor_pb2.FileDescriptorProto()
empty_pb2.DESCRIPTOR.CopyToProto(_empty_fd)
_pool.Add(_empty_fd)
_pool.Add(_build_file())


def _cls(name: str):
    return message_factory.GetMessageClass(_pool.FindMessageTypeByName(name))


Message = _cls("node.Message")
Weights = _cls("node.Weights")
HandShakeRequest = _cls("node.HandShakeRequest")
ResponseMessage = _cls("node.ResponseMessage")
Empty = _cls("google.protobuf.Empty")

SERVICE = "node.NodeServices"
METHODS = {
    "handshake": (HandShakeRequest, ResponseMessage),
    "disconnect": (HandShakeRequest, Empty),
    "send_message": (Message, ResponseMessage),
    "send_weights": (Weights, ResponseMessage),
}


def method_path(name: str) -> str:
    return f"/{SERVICE}/{name}"
