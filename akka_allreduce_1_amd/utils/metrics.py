"""Metrics: counters of every layer plus node metrics, as JSON or Prometheus text.

The reference enables Akka's ClusterMetricsExtension (CPU/heap via Sigar,
application.conf:26-34) but never reads it, and has no application metrics.
Here a registry pulls, on demand, from named sources:

  worker   - WorkerCore stats (messages/bytes in/out, outdated/stale-epoch drops, forced
             catch-ups, duplicates, rounds) and the round-latency histogram (p50/p99)
  master   - rounds started, inits (membership epochs), stale completes
  cluster  - TCP frames/bytes, connects/failures, members up/removed, heartbeats
  comm     - XgmiCommunicator launches / bytes / algorithm split
  plane    - DevicePlane H2D/D2D bytes, kernels, pooled bytes
  node     - CPU %, load average, RSS, threads (psutil), HIP memory when a GPU is in use

`NodeMetricsSampler` is the cluster-metrics-extension analog (periodic node samples).
"""
from __future__ import annotations

import json
import os
import threading
import time
from http.server import BaseHTTPRequestHandler, HTTPServer
from typing import Any, Callable

Source = Callable[[], dict]


def node_metrics() -> dict:
    out: dict[str, Any] = {"pid": os.getpid()}
    try:
        import psutil

        p = psutil.Process()
        mi = p.memory_info()
        out.update(cpu_percent=psutil.cpu_percent(interval=None), rss_bytes=mi.rss, vms_bytes=mi.vms,
                   threads=p.num_threads(), load1=os.getloadavg()[0])
    except Exception:  # noqa: BLE001 - psutil missing or restricted
        out["load1"] = os.getloadavg()[0]
    try:
        import torch

        if torch.cuda.is_initialized():
            d = torch.cuda.current_device()
            out.update(hip_allocated_bytes=torch.cuda.memory_allocated(d),
                       hip_reserved_bytes=torch.cuda.memory_reserved(d))
    except Exception:  # noqa: BLE001
        pass
    return out


def _obj_fields(o: Any) -> dict:
    return {k: getattr(o, k) for k in dir(o) if not k.startswith("_") and isinstance(getattr(o, k), (int, float))}


def worker_source(system, ref) -> Source:
    def f() -> dict:
        st = system.worker_state(ref)
        d = dict(st["stats"])
        d.update({f"latency_{k}": v for k, v in st["round_latency"].items()})
        d.update(round=st["round"], max_round=st["maxRound"], peers=st["numPeers"])
        return d

    return f


def plane_worker_source(system, ref, plane=None) -> Source:
    """A round-plane worker (csrc/runtime/plane_worker.h): protocol counters, round latency
    (fetch -> completion), and the plane's own counters (launches, cold rounds, forces)."""
    def f() -> dict:
        st = system.plane_worker_state(ref)
        d = dict(st["stats"])
        d.update({f"latency_{k}": v for k, v in st["round_latency"].items()})
        d.update(round=st["round"], max_round=st["maxRound"], launched=st["launched"])
        if plane is not None and hasattr(plane, "stats"):
            d.update({f"plane_{k}": v for k, v in _obj_fields(plane.stats).items()})
        return d

    return f


def master_source(system, ref) -> Source:
    return lambda: {k: v for k, v in system.master_state(ref).items() if isinstance(v, (int, float, bool))}


def cluster_source(node) -> Source:
    def f() -> dict:
        d = _obj_fields(node.stats())
        d["members"] = len(node.members())
        return d

    return f


def comm_source(comm) -> Source:
    return lambda: _obj_fields(comm.stats)


def plane_source(plane) -> Source:
    return lambda: {"h2d_bytes": plane.h2d_bytes, "d2d_bytes": plane.d2d_bytes, "kernels": plane.kernels,
                    "cached_bytes": plane.cached_bytes}


def _flatten(prefix: str, d: Any, out: dict) -> None:
    if isinstance(d, dict):
        for k, v in d.items():
            _flatten(f"{prefix}_{k}" if prefix else str(k), v, out)
    elif isinstance(d, bool):
        out[prefix] = int(d)
    elif isinstance(d, (int, float)):
        out[prefix] = d


class MetricsRegistry:
    def __init__(self, labels: dict[str, str] | None = None):
        self.labels = dict(labels or {})
        self._sources: dict[str, Source] = {"node": node_metrics}
        self._lock = threading.Lock()
        self._server: HTTPServer | None = None

    def register(self, name: str, source: Source) -> None:
        with self._lock:
            self._sources[name] = source

    def snapshot(self) -> dict:
        with self._lock:
            items = list(self._sources.items())
        snap: dict[str, Any] = {"ts": time.time(), "labels": self.labels}
        for name, fn in items:
            try:
                snap[name] = fn()
            except Exception as e:  # noqa: BLE001 - a dead source must not kill the exporter
                snap[name] = {"error": repr(e)}
        return snap

    def prometheus_text(self) -> str:
        flat: dict[str, float] = {}
        snap = self.snapshot()
        for k, v in snap.items():
            if k not in ("ts", "labels"):
                _flatten(k, v, flat)
        lab = ",".join(f'{k}="{v}"' for k, v in sorted(self.labels.items()))
        lab = "{" + lab + "}" if lab else ""
        lines = []
        for k, v in sorted(flat.items()):
            name = "mxar_" + "".join(c if c.isalnum() else "_" for c in k)
            lines.append(f"# TYPE {name} gauge")
            lines.append(f"{name}{lab} {float(v)}")
        return "\n".join(lines) + "\n"

    def dump(self, path: str) -> None:
        with open(path, "w") as f:
            json.dump(self.snapshot(), f, indent=1, default=str)

    def serve(self, port: int = 0, host: str = "127.0.0.1") -> int:
        """Serve `/metrics` (Prometheus text) and `/metrics.json`; returns the bound port."""
        reg = self

        class H(BaseHTTPRequestHandler):
            def do_GET(self):  # noqa: N802
                if self.path.startswith("/metrics.json"):
                    body, ctype = json.dumps(reg.snapshot(), default=str).encode(), "application/json"
                elif self.path.startswith("/metrics"):
                    body, ctype = reg.prometheus_text().encode(), "text/plain; version=0.0.4"
                else:
                    self.send_response(404)
                    self.end_headers()
                    return
                self.send_response(200)
                self.send_header("Content-Type", ctype)
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

            def log_message(self, *a):  # quiet
                pass

        self._server = HTTPServer((host, port), H)
        threading.Thread(target=self._server.serve_forever, daemon=True, name="mxar-metrics").start()
        return self._server.server_address[1]

    def close(self) -> None:
        if self._server is not None:
            self._server.shutdown()
            self._server.server_close()
            self._server = None


class NodeMetricsSampler:
    """Samples node metrics every `interval` seconds into a bounded history."""

    def __init__(self, interval: float = 1.0, history: int = 600):
        self.interval = interval
        self.history: list[dict] = []
        self._cap = history
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, daemon=True, name="mxar-node-metrics")

    def start(self) -> "NodeMetricsSampler":
        self._t.start()
        return self

    def _run(self) -> None:
        while not self._stop.wait(self.interval):
            s = node_metrics()
            s["ts"] = time.time()
            self.history.append(s)
            if len(self.history) > self._cap:
                del self.history[: len(self.history) - self._cap]

    def latest(self) -> dict:
        return self.history[-1] if self.history else node_metrics()

    def stop(self) -> None:
        self._stop.set()
        if self._t.is_alive():
            self._t.join(timeout=2 * self.interval + 1)


def write_trace(path: str) -> int:
    """Dump the native tracer's Chrome-trace JSON (chrome://tracing, Perfetto)."""
    from .._native import C

    doc = C.trace.dump_json()
    with open(path, "w") as f:
        f.write(doc)
    return C.trace.size()
