"""Interop with stock reference peers: their ``pickle.dumps([ndarray, ...])`` payload.

Fixtures are written by numpy's own pickler inside the tests (no file from the
reference is loaded).  Decoding is bit-exact; anything but numeric arrays in a
list -- other globals, opcodes, objects -- is rejected without executing it.
"""

from __future__ import annotations

import os
import pickle
import warnings

import numpy as np
import pytest
import torch

from p2pfl_amd.learning.exceptions import DecodingParamsError
from p2pfl_amd.learning.refpickle import decode_reference_payload, encode_reference_payload, looks_like_pickle
from p2pfl_amd.learning.torch_learner import TorchLearner
from p2pfl_amd.learning.wire import decode_params, encode_params
from p2pfl_amd.models import MLP
from p2pfl_amd.settings import Settings


def _learner(seed=0):
    from p2pfl_amd.data import MnistFederatedDM

    return TorchLearner(MLP(seed=seed), MnistFederatedDM(number_sub=200), "me", 1, device=torch.device("cpu"))


@pytest.mark.parametrize("protocol", [2, 3, 4, 5])
def test_reference_payload_decodes_bit_exact(protocol):
    ref = MLP(seed=3)
    blob = pickle.dumps([t.cpu().numpy() for t in ref.state_dict().values()], protocol=protocol)  # what a reference peer sends
    assert looks_like_pickle(blob)
    lrn = _learner()
    params = lrn.decode_parameters(blob)
    for (name, a), b in zip(ref.state_dict().items(), params.values()):
        assert torch.equal(a, b.reshape(a.shape)), name
    lrn.set_parameters(params)
    for a, b in zip(ref.state_dict().values(), lrn.get_parameters().values()):
        assert torch.equal(a, b)


def test_reference_payload_emitted_matches_numpy_pickle():
    lrn = _learner(seed=5)
    old = Settings.WIRE_FORMAT
    Settings.WIRE_FORMAT = "reference"
    try:
        blob = lrn.encode_parameters()
    finally:
        Settings.WIRE_FORMAT = old
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", DeprecationWarning)
        arrays = pickle.loads(blob)  # our own bytes: what a stock reference peer would run
    own = list(lrn.get_parameters().values())
    assert isinstance(arrays, list) and len(arrays) == len(own)
    for a, t in zip(arrays, own):
        assert a.dtype == np.float32 and np.array_equal(a, t.numpy())
    # and it decodes back through the normal path
    back = decode_params(blob)
    assert all(torch.equal(x, y) for x, y in zip(back, own))


def test_reference_payload_keeps_integer_buffers():
    from collections import OrderedDict

    from p2pfl_amd.learning.arena import flatten

    sd = OrderedDict(w=torch.randn(3, 2), n=torch.tensor(7, dtype=torch.int64))
    flat = flatten(sd)
    arrays = pickle.loads(encode_reference_payload(flat))
    assert arrays[1].dtype == np.int64 and int(arrays[1]) == 7


class _Evil:
    def __reduce__(self):
        return (os.system, ("echo pwned",))


@pytest.mark.parametrize(
    "payload",
    [
        pickle.dumps([_Evil()]),
        pickle.dumps({"w": np.zeros(3)}),
        pickle.dumps([np.array([object()], dtype=object)]),
        pickle.dumps([1, 2, 3]),
        pickle.dumps([np.zeros(2)])[:-5],
        b"\x80\x04" + b"garbage",
    ],
)
def test_reference_payload_rejects_everything_else(payload):
    with pytest.raises(DecodingParamsError):
        decode_reference_payload(payload)


def test_count_or_shape_mismatch_is_refused():
    from p2pfl_amd.learning.exceptions import ModelNotMatchingError

    arrays = [t.numpy() for t in MLP(seed=1).state_dict().values()]
    lrn = _learner()
    with pytest.raises(ModelNotMatchingError):
        lrn.decode_parameters(pickle.dumps(arrays[:-1]))  # the reference's zip() would truncate (Q17)
    arrays[0] = arrays[0][:, :10]
    with pytest.raises(ModelNotMatchingError):
        lrn.decode_parameters(pickle.dumps(arrays))


def test_grpc_nodes_federate_on_reference_wire_format():
    from p2pfl_amd.communication.grpc import GrpcCommunicationProtocol
    from p2pfl_amd.data import MnistFederatedDM
    from p2pfl_amd.node import Node
    from p2pfl_amd.utils import check_equal_models, wait_4_results, wait_convergence

    old = Settings.WIRE_FORMAT
    Settings.WIRE_FORMAT = "reference"
    a = Node(MLP(seed=0), MnistFederatedDM(sub_id=0, number_sub=40), protocol=GrpcCommunicationProtocol)
    b = Node(MLP(seed=1), MnistFederatedDM(sub_id=1, number_sub=40), protocol=GrpcCommunicationProtocol)
    a.start()
    b.start()
    try:
        b.connect(a.addr)
        wait_convergence([a, b], 1, only_direct=True)
        a.set_start_learning(rounds=1, epochs=1)
        wait_4_results([a, b], timeout=90)
        check_equal_models([a, b])
    finally:
        Settings.WIRE_FORMAT = old
        a.stop()
        b.stop()
