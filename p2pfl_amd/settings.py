"""Process-global tunables.

Same attribute names and defaults as the reference ``Settings`` class
(reference ``p2pfl/settings.py:26-115``) so user code that mutates them keeps
working.  Periods here are *upper bounds*: the control plane is event driven
(condition variables) and wakes up early when the state it waits on changes,
instead of sleeping a full period like the reference's polling loops.

MI355X-specific knobs (device data plane, kernel selection) are grouped at the
bottom and are new.
"""

from __future__ import annotations


class Settings:
    """Global settings shared by every in-process node (reference quirk Q14)."""

    # ---- general ---------------------------------------------------------
    GRPC_TIMEOUT: float = 10
    """Maximum time (s) to wait for a gRPC request."""
    LOG_LEVEL: str = "INFO"
    """Log level name."""
    LOG_DIR: str = "logs"
    """Directory for the rotating log file."""

    # ---- heartbeat -------------------------------------------------------
    HEARTBEAT_PERIOD: float = 2
    """Period (s) between heartbeats."""
    HEARTBEAT_TIMEOUT: float = 5
    """Silence (s) after which a neighbour is evicted."""

    # ---- gossip ----------------------------------------------------------
    GOSSIP_PERIOD: float = 0.1
    """Period (s) of the control-message relay loop."""
    TTL: int = 10
    """Hop budget of flooded control messages."""
    GOSSIP_MESSAGES_PER_PERIOD: int = 100
    """Relay rate limit: messages per ``GOSSIP_PERIOD``."""
    AMOUNT_LAST_MESSAGES_SAVED: int = 100
    """Size of the duplicate-suppression ring."""
    GOSSIP_MODELS_PERIOD: float = 1
    """Upper bound (s) between two model-gossip iterations."""
    GOSSIP_MODELS_PER_ROUND: int = 2
    """Fan-out of one model-gossip iteration."""
    GOSSIP_EXIT_ON_X_EQUAL_ROUNDS: int = 10
    """Model gossip stops after this many identical status snapshots."""
    GOSSIP_RELAY_GRACE: float | None = None
    """New (exactly-once delivery on a full mesh): when every train-set member
    is a direct neighbour, how long (s) a node lets the ORIGIN of a
    contribution deliver it before relaying it to a peer whose
    ``models_aggregated`` report has not moved (partial-aggregate gossip), and
    how long it lets a train-set neighbour finish its own aggregation before
    diffusing the full model to it -- every model then crosses each link
    once.  Sparser neighbourhoods relay at once, as before.  ``None``: a
    quarter of ``GOSSIP_MODELS_PERIOD``.  0 restores the reference's eager
    re-sends (``gossip_model_stage.py:100-104``, ``train_stage.py:134-139``)."""

    # ---- training --------------------------------------------------------
    ASYNC_DIFFUSION: bool = True
    """Diffuse a round's aggregated model in the background while the next
    round trains (new, on by default; the reference blocks in
    ``GossipModelStage`` until every direct neighbour has the model:
    ``gossip_model_stage.py:84-132``, restored by ``False``).  One immutable
    device snapshot of the aggregate is pushed to every lagging neighbour; a
    newer round's diffusion supersedes an older one."""

    NODE_STREAMS: bool | str = "auto"
    """GPU learners train / evaluate on their own HIP stream, so the
    aggregation and transport work left on the default stream (FedAvg folds of
    arriving models, payload snapshots, the RCCL comm stream's hand-offs) and
    other virtual peers' training overlap a running ``fit()``.  ``"auto"``
    (default) and ``True``: every GPU learner; ``False``: the learner enqueues on
    the caller's stream.  The hand-offs are lazy and event-ordered (the arena's
    ``WeightGuard``): readers of the weights on other streams wait for the last
    write only where they launch, the next write waits for those reads, and a
    lone trainer pays no cross-queue wait at all."""

    EVAL_BATCH_FACTOR: int = 8
    """New: captured evaluation steps (test / validation passes of the graph
    learners) take this many loader batches at once.  Results are the same
    per-sample losses and predictions; the larger launches run at a higher
    MFMA rate.  1 restores the loader's batch."""

    TRAIN_SET_SIZE: int = 4
    """Number of nodes elected to train each experiment."""
    VOTE_TIMEOUT: float = 60
    """Timeout (s) while collecting train-set votes."""
    AGGREGATION_TIMEOUT: float = 300
    """Timeout (s) while waiting for the models of the train set."""
    WAIT_HEARTBEATS_CONVERGENCE: float = 0.2 * HEARTBEAT_TIMEOUT
    """Time (s) to let heartbeats converge before voting."""

    # ---- web / monitoring ------------------------------------------------
    RESOURCE_MONITOR_PERIOD: float = 1
    """Period (s) of the resource monitor."""

    # ---- MI355X data plane (new) ----------------------------------------
    DEVICE_PAYLOADS: bool = True
    """Transports that live in one process hand device-resident flat
    parameter arenas to each other instead of host byte strings."""
    GRPC_MAX_MESSAGE_BYTES: int = 1 << 30
    """gRPC send/receive limit (the reference kept gRPC's 4 MiB default,
    which the 26 MB MNIST CNN exceeds: reference quirk Q6)."""
    WIRE_FORMAT: str = "p2fa"
    """Byte encoding of weights on host transports (gRPC): ``"p2fa"`` (framed,
    checksummed, never executes anything) or ``"reference"`` (the reference's
    ``pickle.dumps([ndarray, ...])``, to federate with stock p2pfl peers; it is
    always *read* with an allow-listed non-executing decoder)."""
    WIRE_DTYPE: str = "fp32"
    """Element type of model arenas on the xGMI data plane: ``"fp32"`` (the
    reference's numerics) or ``"bf16"`` (half the bytes per link; receivers
    average bf16 inputs in fp32)."""
    TORCH_NUM_THREADS: int | None = None
    """If set, ``torch.set_num_threads`` value used by the learners
    (the reference hard-codes 1: ``lightning_learner.py:38``)."""
    TRACE_SPANS: bool = True
    """Record per-stage / per-gossip timing spans in the tracer."""
    CHECKPOINT_DIR: str | None = None
    """If set, every node writes ``<dir>/<addr>/round_<r>.safetensors`` (its
    aggregated model, flat arena + manifest) at the end of each round; see
    :mod:`p2pfl_amd.learning.checkpoint` and ``Node.load_checkpoint``."""
