"""ML-framework-agnostic learner contract (reference ``learning/learner.py:24-150``).

The 11 methods and the constructor signature ``(model, data, self_addr,
epochs)`` are the plug-in point for new training back-ends.  Two optional
methods (with defaults) support the MI355X device data plane:

* :meth:`snapshot_parameters` -- a detached, device-resident flat copy of
  the parameters (what in-process transports ship instead of bytes);
* :meth:`decode_parameters` must accept either wire bytes or such a snapshot.
"""

from __future__ import annotations

from typing import Any, Dict, Optional, Tuple


class NodeLearner:
    def __init__(self, model: Any, data: Any, self_addr: str, epochs: int) -> None:
        raise NotImplementedError

    def set_model(self, model: Any) -> None:
        raise NotImplementedError

    def set_data(self, data: Any) -> None:
        raise NotImplementedError

    def encode_parameters(self, params: Optional[Any] = None) -> bytes:
        raise NotImplementedError

    def decode_parameters(self, data: Any) -> Any:
        raise NotImplementedError

    def set_parameters(self, params: Any) -> None:
        raise NotImplementedError

    def get_parameters(self) -> Any:
        raise NotImplementedError

    def set_epochs(self, epochs: int) -> None:
        raise NotImplementedError

    def fit(self) -> None:
        raise NotImplementedError

    def interrupt_fit(self) -> None:
        raise NotImplementedError

    def evaluate(self) -> Dict[str, float]:
        raise NotImplementedError

    def get_num_samples(self) -> Tuple[int, int]:
        raise NotImplementedError

    # -- optional (device data plane) -------------------------------------
    def snapshot_parameters(self, params: Optional[Any] = None) -> Any:
        """Detached copy suitable for shipping in-process; defaults to bytes."""
        return self.encode_parameters(params)

    # -- optional (asynchronous learners) -----------------------------------
    def evaluate_async(self, on_results: Any = None) -> bool:
        """Enqueue an evaluation whose results reach ``on_results`` later.

        Learners that evaluate synchronously return False and the caller uses
        :meth:`evaluate`."""
        return False

    def drain(self, timeout: Optional[float] = None) -> bool:
        """Wait until the host work of every enqueued pass (metric logging) ran."""
        return True
