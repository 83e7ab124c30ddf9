"""Observability: logger, metric storage, tracer, resource monitor, web client."""

from p2pfl_amd.management.logger import Logger, logger
from p2pfl_amd.management.tracing import Tracer, tracer

__all__ = ["Logger", "logger", "Tracer", "tracer"]
