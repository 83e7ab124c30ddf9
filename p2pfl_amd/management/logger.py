"""Process-wide logger singleton.

API parity with the reference ``Logger`` (``management/logger.py:144-584``):
``info/debug/warning/error/critical(node, msg)``, ``log_metric``,
``log_system_metric``, ``get_local_logs/get_global_logs``,
``register_node/unregister_node``, ``connect_web``, lifecycle hooks and level
helpers, all callable on the class (``logger.info(...)``).

Differences by design:

* Metrics from nodes that are not registered in this process (e.g. received
  from a remote peer) are stored instead of raising (reference quirk Q7); the
  round must then be supplied and the experiment defaults to the receiving
  side's experiment name or ``"experiment"``.
* The file/web handlers run behind a ``QueueListener`` on a thread queue (no
  multiprocessing queue per process).
* A span tracer (:mod:`p2pfl_amd.management.tracing`) is exposed as
  ``logger.tracer`` / ``logger.span(...)``.
"""

from __future__ import annotations

import atexit
import datetime
import logging
import os
import queue
import threading
from logging.handlers import QueueHandler, QueueListener, RotatingFileHandler
from typing import Any, Dict, List, Optional, Tuple

from p2pfl_amd.management.metric_storage import GlobalLogsType, GlobalMetricStorage, LocalLogsType, LocalMetricStorage
from p2pfl_amd.management.node_monitor import NodeMonitor
from p2pfl_amd.management.tracing import tracer as _tracer
from p2pfl_amd.management.web_services import P2pflWebServices
from p2pfl_amd.settings import Settings

GRAY, RED, YELLOW, GREEN, BLUE, CYAN, RESET = (
    "\033[90m",
    "\033[91m",
    "\033[93m",
    "\033[92m",
    "\033[94m",
    "\033[96m",
    "\033[0m",
)
_LEVEL_COLORS = {"DEBUG": BLUE, "INFO": GREEN, "WARNING": YELLOW, "ERROR": RED, "CRITICAL": RED}


class _ColoredFormatter(logging.Formatter):
    def format(self, record: logging.LogRecord) -> str:
        rec = logging.makeLogRecord(record.__dict__)
        color = _LEVEL_COLORS.get(rec.levelname, "")
        rec.levelname = f"{color}{rec.levelname}{RESET}"
        return super().format(rec)


class _WebLogHandler(logging.Handler):
    def __init__(self, web: P2pflWebServices) -> None:
        super().__init__()
        self.web = web

    def emit(self, record: logging.LogRecord) -> None:
        try:
            self.web.send_log(
                datetime.datetime.fromtimestamp(record.created),
                getattr(record, "node", "unknown"),
                record.levelname,
                record.getMessage(),
            )
        except Exception:
            pass


class Logger:
    """Singleton; use the module-level ``logger`` alias (the class itself)."""

    _instance: Optional["Logger"] = None
    _instance_lock = threading.Lock()
    tracer = _tracer

    def __init__(self, p2pfl_web_services: Optional[P2pflWebServices] = None) -> None:
        self.nodes: Dict[str, Tuple[Optional[NodeMonitor], Any]] = {}
        self._nodes_lock = threading.Lock()
        self.local_metrics = LocalMetricStorage()
        self.global_metrics = GlobalMetricStorage()
        self.p2pfl_web_services = p2pfl_web_services

        self.logger = logging.getLogger("p2pfl_amd")
        self.logger.propagate = False
        self.logger.setLevel(logging.getLevelName(Settings.LOG_LEVEL))
        for h in list(self.logger.handlers):
            self.logger.removeHandler(h)

        async_handlers: List[logging.Handler] = []
        if p2pfl_web_services is not None:
            async_handlers.append(_WebLogHandler(p2pfl_web_services))
        try:
            os.makedirs(Settings.LOG_DIR, exist_ok=True)
            fh = RotatingFileHandler(os.path.join(Settings.LOG_DIR, "p2pfl.log"), maxBytes=1_000_000, backupCount=3)
            fh.setFormatter(
                logging.Formatter("[ %(asctime)s | %(node)s | %(levelname)s ]: %(message)s", datefmt="%Y-%m-%d %H:%M:%S")
            )
            async_handlers.append(fh)
        except OSError:
            pass  # read-only cwd: console only

        console = logging.StreamHandler()
        console.setFormatter(
            _ColoredFormatter(
                f"{GRAY}[ {YELLOW}%(asctime)s {GRAY}| {CYAN}%(node)s {GRAY}| %(levelname)s{GRAY} ]:{RESET} %(message)s",
                datefmt="%Y-%m-%d %H:%M:%S",
            )
        )
        self.logger.addHandler(console)

        self._queue: "queue.Queue[logging.LogRecord]" = queue.Queue()
        self.logger.addHandler(QueueHandler(self._queue))
        self.queue_listener = QueueListener(self._queue, *async_handlers)
        self.queue_listener.start()
        atexit.register(self.cleanup)

    # ------------------------------------------------------------------
    # singleton management
    # ------------------------------------------------------------------
    @classmethod
    def get_instance(cls) -> "Logger":
        if cls._instance is None:
            with cls._instance_lock:
                if cls._instance is None:
                    cls._instance = Logger()
        return cls._instance

    @classmethod
    def connect_web(cls, url: str, key: str) -> None:
        with cls._instance_lock:
            if cls._instance is not None:
                cls._instance.queue_listener.stop()
            cls._instance = Logger(p2pfl_web_services=P2pflWebServices(url, key))

    def cleanup(self) -> None:
        for node in list(self.nodes):
            try:
                Logger.unregister_node(node)
            except Exception:
                pass
        try:
            self.queue_listener.stop()
        except Exception:
            pass

    # ------------------------------------------------------------------
    # levels
    # ------------------------------------------------------------------
    @staticmethod
    def set_level(level: Any) -> None:
        if isinstance(level, str):
            level = logging.getLevelName(level)
        Logger.get_instance().logger.setLevel(level)

    @staticmethod
    def get_level() -> int:
        return Logger.get_instance().logger.getEffectiveLevel()

    @staticmethod
    def get_level_name(lvl: int) -> str:
        return logging.getLevelName(lvl)

    # ------------------------------------------------------------------
    # application logging
    # ------------------------------------------------------------------
    def log(self, level: int, node: str, message: str) -> None:
        if level not in (logging.DEBUG, logging.INFO, logging.WARNING, logging.ERROR, logging.CRITICAL):
            raise ValueError(f"Invalid level: {level}")
        self.logger.log(level, message, extra={"node": node})

    @staticmethod
    def debug(node: str, message: str) -> None:
        Logger.get_instance().log(logging.DEBUG, node, message)

    @staticmethod
    def info(node: str, message: str) -> None:
        Logger.get_instance().log(logging.INFO, node, message)

    @staticmethod
    def warning(node: str, message: str) -> None:
        Logger.get_instance().log(logging.WARNING, node, message)

    @staticmethod
    def error(node: str, message: str) -> None:
        Logger.get_instance().log(logging.ERROR, node, message)

    @staticmethod
    def critical(node: str, message: str) -> None:
        Logger.get_instance().log(logging.CRITICAL, node, message)

    # ------------------------------------------------------------------
    # metrics
    # ------------------------------------------------------------------
    @staticmethod
    def log_metric(
        node: str,
        metric: str,
        value: float,
        step: Optional[int] = None,
        round: Optional[int] = None,
        exp: Optional[str] = None,
    ) -> None:
        inst = Logger.get_instance()
        entry = inst.nodes.get(node)
        state = entry[1] if entry is not None else None
        if round is None:
            round = getattr(state, "round", None)
        if round is None:
            raise Exception("No round provided. Needed for training metrics.")
        if exp is None:
            exp = getattr(state, "actual_exp_name", None) or "experiment"
        value = float(value)
        if step is None:
            inst.global_metrics.add_log(exp, round, metric, node, value)
        else:
            inst.local_metrics.add_log(exp, round, metric, node, value, step)
        web = inst.p2pfl_web_services
        if web is not None:
            try:
                if step is None:
                    web.send_global_metric(exp, round, metric, node, value)
                else:
                    web.send_local_metric(exp, round, metric, node, value, step)
            except Exception:
                pass

    @staticmethod
    def log_system_metric(node: str, metric: str, value: float, time: datetime.datetime) -> None:
        web = Logger.get_instance().p2pfl_web_services
        if web is not None:
            try:
                web.send_system_metric(node, metric, value, time)
            except Exception:
                pass

    @staticmethod
    def get_local_logs() -> LocalLogsType:
        return Logger.get_instance().local_metrics.get_all_logs()

    @staticmethod
    def get_global_logs() -> GlobalLogsType:
        return Logger.get_instance().global_metrics.get_all_logs()

    # ------------------------------------------------------------------
    # node registration
    # ------------------------------------------------------------------
    @staticmethod
    def register_node(node: str, state: Any, simulation: bool) -> None:
        inst = Logger.get_instance()
        with inst._nodes_lock:
            if node in inst.nodes:
                raise Exception(f"Node {node} already registered.")
            monitor = None
            if inst.p2pfl_web_services is not None:
                try:
                    inst.p2pfl_web_services.register_node(node, simulation)
                    monitor = NodeMonitor(node, Logger.log_system_metric)
                    monitor.start()
                except Exception as e:
                    inst.log(logging.WARNING, node, f"web registration failed: {e}")
            inst.nodes[node] = (monitor, state)

    @staticmethod
    def unregister_node(node: str) -> None:
        inst = Logger.get_instance()
        with inst._nodes_lock:
            if node not in inst.nodes:
                raise KeyError(f"Node {node} not registered.")
            monitor, _ = inst.nodes.pop(node)
        if monitor is not None:
            monitor.stop()
        if inst.p2pfl_web_services is not None:
            inst.p2pfl_web_services.unregister_node(node)

    # ------------------------------------------------------------------
    # lifecycle hooks
    # ------------------------------------------------------------------
    @staticmethod
    def experiment_started(node: str) -> None:
        Logger.debug(node, "Experiment started")

    @staticmethod
    def experiment_finished(node: str) -> None:
        Logger.debug(node, "Experiment finished")

    @staticmethod
    def round_finished(node: str) -> None:
        entry = Logger.get_instance().nodes.get(node)
        r = getattr(entry[1], "round", None) if entry else None
        Logger.debug(node, f"Round {r} finished")

    # ------------------------------------------------------------------
    # tracing
    # ------------------------------------------------------------------
    @staticmethod
    def span(node: str, name: str, **attrs: Any):
        return _tracer.span(node, name, **attrs)


logger = Logger
