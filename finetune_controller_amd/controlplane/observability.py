"""Prometheus metrics for the control plane (the reference has none: SURVEY.md §5.5 "No Prometheus /
metrics endpoint").

* API: request count and latency per method / route TEMPLATE (``/api/v1/jobs/{job_id}``, never the
  raw path, so cardinality stays bounded) / status, jobs submitted per model and device, submit
  failures per HTTP status.  Scraped at ``GET /metrics`` (outside ``/api/v1``: no auth, like
  ``/health``).
* Monitor: reconcile passes, their duration and errors, leadership, PyTorchJobs seen per mapped
  status, Kueue-pending workloads.  The API process exposes them when it runs the monitor in-process
  (``DEV_LOCAL_JOB_MONITOR``); the standalone monitor serves them on ``MONITOR_METRICS_PORT``.

Each AppContext owns its own ``CollectorRegistry`` (several apps in one process -- tests -- never
collide).  With several uvicorn workers set ``PROMETHEUS_MULTIPROC_DIR``: ``/metrics`` then
aggregates every worker's counters through prometheus_client's multiprocess collector.
"""
from __future__ import annotations

import os
import time

from prometheus_client import CONTENT_TYPE_LATEST, CollectorRegistry, Counter, Gauge, Histogram, generate_latest

_LAT_BUCKETS = (0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1.0, 2.5, 5.0, 10.0)


class ControlPlaneMetrics:
    def __init__(self, registry: CollectorRegistry | None = None):
        self.registry = registry or CollectorRegistry()
        r = self.registry
        self.http_requests = Counter("ftc_http_requests", "HTTP requests served", ["method", "route", "status"],
                                     registry=r)
        self.http_latency = Histogram("ftc_http_request_duration_seconds", "HTTP request latency",
                                      ["method", "route"], buckets=_LAT_BUCKETS, registry=r)
        self.jobs_submitted = Counter("ftc_jobs_submitted", "Fine-tune jobs accepted by POST /api/v1/jobs",
                                      ["model", "device"], registry=r)
        self.submit_failures = Counter("ftc_job_submit_failures", "Rejected or failed job submissions",
                                       ["status"], registry=r)
        self.reconcile_passes = Counter("ftc_monitor_reconcile_passes", "Monitor reconcile passes", registry=r)
        self.reconcile_errors = Counter("ftc_monitor_reconcile_errors", "Monitor passes that raised", registry=r)
        self.reconcile_seconds = Histogram("ftc_monitor_reconcile_seconds", "Duration of one reconcile pass",
                                           buckets=_LAT_BUCKETS, registry=r)
        self.jobs_updated = Counter("ftc_monitor_job_updates", "Job documents updated by the monitor", registry=r)
        self.is_leader = Gauge("ftc_monitor_is_leader", "1 while this process holds the monitor lease", registry=r)
        self.cluster_jobs = Gauge("ftc_cluster_jobs", "PyTorchJobs in the namespace by mapped status", ["status"],
                                  registry=r)
        self.kueue_pending = Gauge("ftc_kueue_pending_workloads", "Kueue workloads waiting for quota", registry=r)
        self._seen_status: set[str] = set()

    def exposition(self) -> tuple[bytes, str]:
        if os.environ.get("PROMETHEUS_MULTIPROC_DIR"):
            from prometheus_client import multiprocess

            reg = CollectorRegistry()
            multiprocess.MultiProcessCollector(reg)
            return generate_latest(reg), CONTENT_TYPE_LATEST
        return generate_latest(self.registry), CONTENT_TYPE_LATEST

    def observe_pass(self, t0: float, by_status: dict[str, int], pending: int, updated: int):
        self.reconcile_passes.inc()
        self.reconcile_seconds.observe(time.perf_counter() - t0)
        for st in list(self._seen_status):
            if st not in by_status:
                self.cluster_jobs.labels(st).set(0)
        for st, n in by_status.items():
            self.cluster_jobs.labels(st).set(n)
            self._seen_status.add(st)
        self.kueue_pending.set(pending)
        self.jobs_updated.inc(updated)


def get_metrics(ctx) -> ControlPlaneMetrics:
    """The context's metrics (created on first use)."""
    m = getattr(ctx, "_metrics", None)
    if m is None:
        m = ControlPlaneMetrics()
        object.__setattr__(ctx, "_metrics", m)
    return m


_METHODS = frozenset({"GET", "POST", "PUT", "PATCH", "DELETE", "HEAD", "OPTIONS"})


class PrometheusMiddleware:
    """Pure ASGI: counts HTTP requests by method / route template / status and times them."""

    def __init__(self, app, metrics: ControlPlaneMetrics):
        self.app = app
        self.m = metrics

    async def __call__(self, scope, receive, send):
        if scope["type"] != "http":
            return await self.app(scope, receive, send)
        t0 = time.perf_counter()
        status = {"code": 500}

        async def _send(msg):
            if msg["type"] == "http.response.start":
                status["code"] = msg["status"]
            await send(msg)

        try:
            await self.app(scope, receive, _send)
        finally:
            route = getattr(scope.get("route"), "path", None) or "<unmatched>"
            method = scope.get("method", "?")
            if method not in _METHODS:  # the request line is client text: keep the label set closed
                method = "OTHER"
            self.m.http_requests.labels(method, route, str(status["code"])).inc()
            self.m.http_latency.labels(method, route).observe(time.perf_counter() - t0)
