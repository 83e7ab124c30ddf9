"""REST client for the p2pfl-web dashboard.

Endpoints and payload fields follow the reference client
(``management/p2pfl_web_services.py:68-265``): ``/node``, ``/node-log``,
``/node-metric/{local,global,system}`` with an ``x-api-key`` header.  Uses only
the standard library (``urllib``) so no extra dependency is needed.
"""

from __future__ import annotations

import datetime
import json
import urllib.error
import urllib.request
from typing import Any, Dict, Optional


class P2pflWebServicesError(Exception):
    def __init__(self, code: int, message: str) -> None:
        self.code = code
        self.message = message
        super().__init__(f"Error {code}: {message}")


class P2pflWebServices:
    def __init__(self, url: str, key: str, timeout: float = 5.0) -> None:
        if not url.startswith("https://"):
            print("P2pflWebServices Warning: Connection must be over https, traffic will not be encrypted")
        self._url = url.rstrip("/")
        self._key = key
        self.timeout = timeout
        self.node_id: Dict[str, Any] = {}

    # -- transport -----------------------------------------------------
    def _post(self, path: str, data: Dict[str, Any]) -> Any:
        req = urllib.request.Request(
            self._url + path,
            data=json.dumps(data, default=str).encode(),
            headers={"Content-Type": "application/json", "x-api-key": self._key},
            method="POST",
        )
        try:
            with urllib.request.urlopen(req, timeout=self.timeout) as resp:
                body = resp.read()
                return json.loads(body) if body else {}
        except urllib.error.HTTPError as e:
            raise P2pflWebServicesError(e.code, e.read().decode(errors="replace")) from e
        except urllib.error.URLError as e:
            raise P2pflWebServicesError(-1, str(e)) from e

    def _nid(self, node: str) -> Any:
        if node not in self.node_id:
            raise ValueError(f"Node {node} not registered")
        return self.node_id[node]

    # -- API -----------------------------------------------------------
    def register_node(self, node: str, is_simulated: bool) -> None:
        res = self._post(
            "/node",
            {
                "address": node,
                "is_simulated": is_simulated,
                "creation_date": datetime.datetime.now().strftime("%Y-%m-%d %H:%M:%S"),
            },
        )
        self.node_id[node] = res.get("node_id")

    def unregister_node(self, node: str) -> None:
        self.node_id.pop(node, None)

    def send_log(self, time: datetime.datetime, node: str, level: str, message: str) -> None:
        self._post(
            "/node-log",
            {"time": time.strftime("%Y-%m-%d %H:%M:%S"), "node_id": self._nid(node), "level": level, "message": message},
        )

    def send_local_metric(self, exp: str, round: int, metric: str, node: str, value: float, step: int) -> None:
        self._post(
            "/node-metric/local",
            {"node_id": self._nid(node), "exp_id": exp, "metric_name": metric, "round": round, "step": step, "value": value},
        )

    def send_global_metric(self, exp: str, round: int, metric: str, node: str, value: float) -> None:
        self._post(
            "/node-metric/global",
            {"node_id": self._nid(node), "exp_id": exp, "metric_name": metric, "round": round, "value": value},
        )

    def send_system_metric(self, node: str, metric: str, value: float, time: datetime.datetime) -> None:
        self._post(
            "/node-metric/system",
            {"node_id": self._nid(node), "metric_name": metric, "time": time.strftime("%Y-%m-%d %H:%M:%S"), "value": value},
        )

    def get_pending_actions(self) -> Optional[list]:
        return None
