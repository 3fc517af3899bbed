"""Prometheus metrics of the control plane (controlplane/observability.py): route-template request
counters, submissions per model/device, submit failures, and the monitor's per-pass gauges."""
from fastapi.testclient import TestClient
from prometheus_client.parser import text_string_to_metric_families

from finetune_controller_amd.controlplane.api.app import create_app
from finetune_controller_amd.controlplane.context import AppContext


def _samples(text):
    out = {}
    for fam in text_string_to_metric_families(text):
        for s in fam.samples:
            out[(s.name, tuple(sorted(s.labels.items())))] = s.value
    return out


def test_metrics_endpoint_counts_api_and_monitor(tmp_path):
    ctx = AppContext.local(workdir=str(tmp_path), run_processes=False)
    app = create_app(ctx, run_monitor=False, force_auth=False)
    with TestClient(app) as c:
        ids = []
        for i in range(2):
            r = c.post("/api/v1/jobs", data={"job_name": f"j{i}", "model": "Llama3-8B-LoRA", "device": "mi355x",
                                            "task": "causal_lm", "user_id": "alice"})
            ids.append(r.json()["job_id"])
        assert c.post("/api/v1/jobs", data={"job_name": "x", "model": "Nope", "device": "mi355x",
                                           "task": "causal_lm", "user_id": "alice"}).status_code == 404
        for jid in ids:
            assert c.get(f"/api/v1/jobs/{jid}").status_code == 200
        for _ in range(3):
            ctx.kube.reconcile()
        mon = app.state.monitor
        c.portal.call(mon.reconcile_once)
        for verb in ("FROB", "XYZZY"):  # arbitrary request-line methods share one label value
            c.request(verb, "/api/v1/health")
        text = c.get("/metrics").text
    s = _samples(text)
    assert s[("ftc_jobs_submitted_total", (("device", "mi355x"), ("model", "Llama3-8B-LoRA")))] == 2
    assert s[("ftc_job_submit_failures_total", (("status", "404"),))] == 1
    # one series per route TEMPLATE, not per job id
    get_job = ("ftc_http_requests_total", (("method", "GET"), ("route", "/api/v1/jobs/{job_id}"), ("status", "200")))
    assert s[get_job] == 2
    assert not any("alice" in dict(k[1]).get("route", "") or ids[0] in dict(k[1]).get("route", "") for k in s)
    assert s[("ftc_monitor_reconcile_passes_total", ())] == 1
    running = sum(v for (n, lab), v in s.items() if n == "ftc_cluster_jobs")
    assert running == 2
    methods = {dict(k[1]).get("method") for k in s if k[0] == "ftc_http_requests_total"}
    assert "OTHER" in methods and not methods & {"FROB", "XYZZY"}
