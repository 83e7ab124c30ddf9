"""Per-node resource monitor (reference ``management/node_monitor.py:30-86``).

Samples CPU %, RAM %, network MB/s and -- new on MI355X -- the GPU's
allocated / reserved HBM of the current process every
``Settings.RESOURCE_MONITOR_PERIOD`` seconds and reports them through a
callback (the logger forwards them to the web services).
"""

from __future__ import annotations

import datetime
import threading
from typing import Callable, Dict, Optional

from p2pfl_amd.settings import Settings

try:  # psutil is optional
    import psutil  # type: ignore
except Exception:  # pragma: no cover
    psutil = None


class NodeMonitor(threading.Thread):
    def __init__(
        self,
        node_addr: str,
        metric_report_callback: Callable[[str, str, float, datetime.datetime], None],
        period: Optional[float] = None,
    ) -> None:
        super().__init__(name=f"resource-monitor-thread-{node_addr}", daemon=True)
        self.node_addr = node_addr
        self.metric_report_callback = metric_report_callback
        self.period = Settings.RESOURCE_MONITOR_PERIOD if period is None else period
        self._stop_evt = threading.Event()
        self._last_net: Optional[tuple] = None

    def stop(self) -> None:
        self._stop_evt.set()

    def run(self) -> None:
        while not self._stop_evt.is_set():
            now = datetime.datetime.now()
            for key, value in self.sample().items():
                self.metric_report_callback(self.node_addr, key, value, now)
            self._stop_evt.wait(self.period)

    def sample(self) -> Dict[str, float]:
        res: Dict[str, float] = {}
        if psutil is not None:
            res["cpu"] = float(psutil.cpu_percent())
            res["ram"] = float(psutil.virtual_memory().percent)
            net = psutil.net_io_counters()
            if self._last_net is not None:
                res["net_in"] = (net.bytes_recv - self._last_net[0]) / self.period / 2**20
                res["net_out"] = (net.bytes_sent - self._last_net[1]) / self.period / 2**20
            self._last_net = (net.bytes_recv, net.bytes_sent)
        try:
            import torch

            if torch.cuda.is_available():
                res["gpu_mem_alloc_gb"] = torch.cuda.memory_allocated() / 2**30
                res["gpu_mem_reserved_gb"] = torch.cuda.memory_reserved() / 2**30
        except Exception:
            pass
        return res
