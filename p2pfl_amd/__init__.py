"""p2pfl_amd -- a decentralized federated-learning engine built for AMD MI355X.

Same capabilities and user-facing API as p2pfl (``Node``, ``NodeLearner``,
aggregator plug-ins, the vote -> train -> gossip -> aggregate stage machine,
in-memory and gRPC transports), re-designed MI355X-first: flat parameter
arenas, hand-written HIP/CDNA4 kernels for aggregation, optimizers and the
MNIST CNN training step, device-resident gossip payloads, and RCCL/xGMI for
one-peer-per-GPU deployments.
"""

__version__ = "0.1.0"

from p2pfl_amd.settings import Settings  # noqa: E402

__all__ = ["Settings", "__version__"]
