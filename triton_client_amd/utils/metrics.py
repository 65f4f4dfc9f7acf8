"""Prometheus observability (reference: ``data/prometheus.yml`` scrapes Triton
on :8002 and the client's evaluation exporter on :7658 —
``communicator/evaluate_inference.py:52-61``).

* :class:`ServerMetrics` — Triton metric names (nv_inference_request_success,
  nv_inference_request_failure, nv_inference_count, nv_inference_exec_count,
  nv_inference_request_duration_us) so existing Grafana dashboards work.
* :class:`ClientMetrics` — frames_total, per-stage latency histograms, FPS,
  RPC bytes, DP queue depth.
* :class:`EvalMetrics`  — the reference's Summary names: precision, recall,
  ap, fone, ap_class.

All exporters share one process-wide registry per port; ``port=None`` keeps
the metrics in-process (tests) without starting an HTTP server.
"""
from __future__ import annotations

import threading
import time
from typing import Dict, Optional

try:
    from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram, Summary, start_http_server
    HAVE_PROM = True
except ImportError:  # pragma: no cover
    HAVE_PROM = False

_STARTED: Dict[int, CollectorRegistry] = {}
_LOCK = threading.Lock()


def _registry(port: Optional[int]):
    if not HAVE_PROM:
        return None
    if port is None:
        return CollectorRegistry()
    with _LOCK:
        if port not in _STARTED:
            reg = CollectorRegistry()
            start_http_server(port, registry=reg)
            _STARTED[port] = reg
        return _STARTED[port]


class ServerMetrics:
    def __init__(self, port: Optional[int] = 8002):
        self.reg = _registry(port)
        if self.reg is None:
            return
        lab = ["model", "version"]
        self.success = Counter("nv_inference_request_success", "successful inference requests", lab, registry=self.reg)
        self.failure = Counter("nv_inference_request_failure", "failed inference requests", lab, registry=self.reg)
        self.count = Counter("nv_inference_count", "inferences performed", lab, registry=self.reg)
        self.exec_count = Counter("nv_inference_exec_count", "model executions", lab, registry=self.reg)
        self.duration = Counter("nv_inference_request_duration_us", "cumulative request duration (us)", lab,
                                registry=self.reg)

    def request(self, model: str, ok: bool, seconds: float, version: str = "1") -> None:
        if self.reg is None:
            return
        (self.success if ok else self.failure).labels(model, version).inc()
        if ok:
            self.count.labels(model, version).inc()
            self.exec_count.labels(model, version).inc()
        self.duration.labels(model, version).inc(seconds * 1e6)


class ClientMetrics:
    STAGES = ("decode", "preprocess", "infer", "postprocess", "publish", "total")

    def __init__(self, port: Optional[int] = None, prefix: str = "tca_client"):
        self.reg = _registry(port)
        self._t0 = time.perf_counter()
        self._frames = 0
        if self.reg is None:
            return
        self.frames = Counter(f"{prefix}_frames_total", "frames processed", registry=self.reg)
        self.latency = Histogram(f"{prefix}_stage_latency_seconds", "per-stage latency", ["stage"],
                                 buckets=(1e-4, 3e-4, 1e-3, 3e-3, 1e-2, 3e-2, 0.1, 0.3, 1.0), registry=self.reg)
        self.fps = Gauge(f"{prefix}_fps", "frames per second since start", registry=self.reg)
        self.rpc_bytes = Counter(f"{prefix}_rpc_bytes_total", "bytes sent+received over gRPC", registry=self.reg)
        self.queue_depth = Gauge(f"{prefix}_dp_queue_depth", "frames waiting per GPU", ["rank"], registry=self.reg)

    def stage(self, name: str, seconds: float) -> None:
        if self.reg is not None:
            self.latency.labels(name).observe(seconds)

    def frame(self, n: int = 1) -> None:
        self._frames += n
        if self.reg is not None:
            self.frames.inc(n)
            self.fps.set(self._frames / max(time.perf_counter() - self._t0, 1e-9))

    def bytes(self, n: int) -> None:
        if self.reg is not None:
            self.rpc_bytes.inc(n)


class EvalMetrics:
    """Same metric names as the reference evaluator (evaluate_inference.py:57-61)."""

    def __init__(self, port: Optional[int] = 7658):
        self.reg = _registry(port)
        if self.reg is None:
            return
        self.p_summary = Summary("precision", "precision per class", registry=self.reg)
        self.r_summary = Summary("recall", "recall per class", registry=self.reg)
        self.ap_summary = Summary("ap", "average precision per class", registry=self.reg)
        self.f1_summary = Summary("fone", "F1 per class", registry=self.reg)
        self.ap_class_summary = Summary("ap_class", "classes with AP", registry=self.reg)


class StageTimer:
    """with timer('preprocess'): ... → ClientMetrics.stage() + a roctx range of
    the same name (utils/trace.py)."""

    def __init__(self, metrics: Optional[ClientMetrics]):
        self.m = metrics

    def __call__(self, name: str):
        return _Ctx(self.m, name)


class _Ctx:
    def __init__(self, m, name):
        self.m, self.name = m, name

    def __enter__(self):
        from .trace import push
        push(self.name)
        self.t = time.perf_counter()
        return self

    def __exit__(self, *exc):
        from .trace import pop
        pop()
        if self.m is not None:
            self.m.stage(self.name, time.perf_counter() - self.t)
