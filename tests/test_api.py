"""Every route of the REST + WebSocket surface against in-process fakes: in-memory
Mongo engine, local object store, FakeCluster (simulated pods) -- SURVEY.md §4 "[new] API integration"."""
import asyncio
import io
import json
import zipfile

import httpx
import pytest
from fastapi.testclient import TestClient

from finetune_controller_amd.controlplane.api.app import create_app
from finetune_controller_amd.controlplane.context import AppContext
from finetune_controller_amd.controlplane.monitor.reconciler import JobMonitor
from finetune_controller_amd.controlplane.tasks import services

FORM = {"job_name": "my run", "model": "Llama3-8B-LoRA", "device": "mi355x", "task": "causal_lm",
        "arguments": json.dumps({"max_steps": 3, "lora_r": 8})}


@pytest.fixture
def env(tmp_path):
    ctx = AppContext.local(workdir=str(tmp_path), run_processes=False)
    ctx.kube.sim_ticks = 2
    app = create_app(ctx, run_monitor=False, force_auth=False)
    with TestClient(app) as c:
        yield ctx, c


def settle(ctx, rounds=12):
    """Drive the FakeCluster and one monitor pass per round (sidecar threads get time to sync)."""
    import time

    mon = JobMonitor(ctx, interval=0)
    ctx.kube.sync_interval = 0.02
    for i in range(rounds * 10):
        ctx.kube.reconcile()
        asyncio.run(mon.reconcile_once())
        time.sleep(0.03)
        if i >= rounds and not ctx.kube.list_pytorchjobs(ctx.namespace):
            break


def submit(c, **over):
    f = dict(FORM)
    f.update(over)
    r = c.post("/api/v1/jobs", data=f)
    assert r.status_code == 200, r.text
    return r.json()["job_id"]


def test_health_models_details(env):
    ctx, c = env
    assert c.get("/health").json() == {"status": "ok"}
    assert c.get("/api/v1/health").json() == {"status": "ok"}
    models = c.get("/api/v1/models").json()
    assert "Llama3-8B-LoRA" in models
    m = models["Llama3-8B-LoRA"]
    assert m["devices"] == ["cpu", "mi355x"] and "lora_r" in m["arguments"] and m["task"] == "causal_lm"
    d = c.get("/api/v1/models/Llama3-8B-LoRA").json()
    assert d["task"] == "causal_lm" and d["framework"] == "pytorch"
    assert d["arguments"]["accelerator_count"] == 1 and "image" not in d["arguments"]
    assert c.get("/api/v1/models/Nope").status_code == 404
    assert c.get("/api/v1/sample-data.csv").text.startswith("Id,SMILES,esol")


def test_submit_validation_errors(env):
    ctx, c = env
    assert c.post("/api/v1/jobs", data={"job_name": "x"}).status_code == 422
    assert c.post("/api/v1/jobs", data=dict(FORM, device="tpu")).status_code == 422
    assert c.post("/api/v1/jobs", data=dict(FORM, arguments="{bad")).json()["detail"] == "Invalid JSON for arguments"
    r = c.post("/api/v1/jobs", data=dict(FORM, arguments=json.dumps({"lora_r": 0})))
    assert r.status_code == 400 and "Invalid model parameters" in r.json()["detail"] and "lora_r" in r.json()["detail"]
    r = c.post("/api/v1/jobs", data=dict(FORM, task="regression"))
    assert r.status_code == 400 and "Invalid task" in r.json()["detail"]
    assert c.post("/api/v1/jobs", data=dict(FORM, model="Nope")).status_code == 404
    assert c.post("/api/v1/jobs", data=dict(FORM, user_id="a!")).status_code == 422
    for bad in ("ftp://h/x.csv", "not a url", "http:///nohost"):  # (submit is rate limited to 10/min)
        r = c.post("/api/v1/jobs", data=dict(FORM, dataset_url=bad))
        assert r.status_code == 422 and "dataset_url" in r.json()["detail"], bad
    # a malformed row-index filter is the client's error, not a server failure
    for path in ("/api/v1/jobs", "/api/v1/datasets"):
        r = c.get(path, params={"limit": "1,two"})
        assert r.status_code == 422 and "limit" in r.json()["detail"], path
    assert c.get("/api/v1/jobs", params={"limit": "1,2"}).status_code == 200


def test_dataset_url_into_the_cluster_network_is_refused(env):
    """The API server fetches dataset_url itself: the cloud metadata endpoint is not a dataset."""
    ctx, c = env
    r = c.post("/api/v1/jobs", data=dict(FORM, dataset_url="http://169.254.169.254/latest/meta-data/"))
    assert r.status_code == 422 and "non-public" in r.json()["detail"]
    assert ctx.kube.list_pytorchjobs(ctx.namespace) == []


def test_submit_lifecycle_metrics_logs_cancel(env):
    ctx, c = env
    jid = submit(c)
    j = c.get(f"/api/v1/jobs/{jid}").json()
    assert j["status"] == "queued" and j["arguments"]["lora_r"] == 8 and j["atrifacts_uri"].endswith(f"{jid}/artifacts")
    assert c.get(f"/api/v1/jobs/{jid}/metrics").status_code == 202  # running, no metrics yet
    settle(ctx)
    j = c.get(f"/api/v1/jobs/{jid}").json()
    assert j["status"] == "completed" and j["metadata"]["training_duration"] >= 0
    assert j["metadata"]["completion_time"] and j["duration"] is not None
    m = c.get(f"/api/v1/jobs/{jid}/metrics").json()
    steps = [row["step"] for row in m["metrics"]]
    assert steps == sorted(steps, reverse=True) and m["metrics_url"]
    # succeeded PyTorchJobs are deleted by the monitor
    assert c.get("/api/v1/admin/jobs/list").json() == {"jobs": []}
    assert c.post(f"/api/v1/jobs/{jid}/cancel").status_code == 409
    jid2 = submit(c)
    r = c.post(f"/api/v1/jobs/{jid2}/cancel").json()
    assert r["status"] == "canceled" and r["end_time"]
    assert c.get(f"/api/v1/jobs/{jid2}").json()["metadata"]["message"] == "Job canceled by user"
    page = c.get("/api/v1/jobs", params={"page": 1, "page_size": 10}).json()
    assert page["total"] == 2 and {i["status"] for i in page["items"]} == {"completed", "canceled"}
    item = [i for i in page["items"] if i["job_id"] == jid][0]
    assert item["meta_"]["data"]["promotion_path"] == "language/llama3-8b/lora" and item["index_"] >= 1


def test_monitor_retries_a_failed_delete_of_a_succeeded_job(env, monkeypatch):
    """The reference deletes a succeeded PyTorchJob once; if that call fails, the job is already
    'completed' in the DB and a status-only reconciler would leave it on the cluster for good."""
    ctx, c = env
    jid = submit(c)
    real = ctx.kube.delete_pytorchjob
    calls = []

    def flaky(ns, name):
        calls.append(name)
        if len(calls) == 1:
            raise RuntimeError("apiserver unavailable")
        return real(ns, name)

    monkeypatch.setattr(ctx.kube, "delete_pytorchjob", flaky)
    settle(ctx)
    assert c.get(f"/api/v1/jobs/{jid}").json()["status"] == "completed"
    assert calls[:2] == [jid, jid] and ctx.kube.list_pytorchjobs(ctx.namespace) == []


def test_monitor_keeps_its_lease_through_a_slow_pass(env):
    """A reconcile pass longer than the lease TTL renews the lease as it runs: a second monitor cannot
    take over mid-pass and act on the same jobs."""
    from finetune_controller_amd.controlplane.monitor.reconciler import LEASE

    ctx, _ = env
    mon = JobMonitor(ctx, interval=0, lease_ttl=0.3)

    async def slow_pass():
        await asyncio.sleep(1.0)  # > 3 x the TTL
        return 0

    mon.reconcile_once = slow_pass

    async def scenario():
        assert await ctx.store.acquire_lock(LEASE, mon.owner, mon.lease_ttl)
        passing = asyncio.create_task(mon._reconcile_holding_lease())
        taken = []
        for _ in range(8):
            await asyncio.sleep(0.1)
            taken.append(await ctx.store.acquire_lock(LEASE, "other-replica", 0.3))
        await passing
        return taken

    assert not any(asyncio.run(scenario()))


@pytest.mark.parametrize("renewal", ["raises", "lost"])
def test_monitor_stops_writing_once_its_lease_lapses(env, monkeypatch, renewal):
    """a pass whose lease renewals fail (the lease lapses at the last good renewal's expiry) or
    whose renewal finds the lease taken makes no further status writes or deletes in that pass."""
    import time as _time

    from finetune_controller_amd.controlplane.monitor.reconciler import LEASE

    ctx, c = env
    jid = submit(c)
    ctx.kube.reconcile()
    real_list = ctx.kube.list_pytorchjobs

    def slow_list(ns):
        _time.sleep(0.8)  # > the 0.3 s TTL: the lease is gone when the pass reaches its first write
        return real_list(ns)

    monkeypatch.setattr(ctx.kube, "list_pytorchjobs", slow_list)
    mon = JobMonitor(ctx, interval=0, lease_ttl=0.3)
    real_acquire = ctx.store.acquire_lock

    async def acquire(name, owner, ttl):
        if owner == mon.owner and renewal == "raises":
            raise RuntimeError("mongo unreachable")
        if owner == mon.owner:  # "lost": another replica holds it now
            return False
        return await real_acquire(name, owner, ttl)

    writes = []
    real_update = ctx.store.update_job_status

    async def update(*a, **k):
        writes.append(a[0])
        return await real_update(*a, **k)

    async def scenario():
        assert await real_acquire(LEASE, mon.owner, mon.lease_ttl)
        monkeypatch.setattr(ctx.store, "acquire_lock", acquire)
        monkeypatch.setattr(ctx.store, "update_job_status", update)
        await mon._reconcile_holding_lease()

    asyncio.run(scenario())
    assert writes == [], writes
    assert c.get(f"/api/v1/jobs/{jid}").json()["status"] == "queued"


def test_monitor_fails_a_job_whose_pytorchjob_vanished(env):
    """A PyTorchJob deleted behind the controller's back (kubectl, a cluster reset) must not leave its
    job 'running' in the UI forever: after the grace period the monitor marks it failed."""
    ctx, c = env
    jid = submit(c)
    keep = submit(c)
    mon = JobMonitor(ctx, interval=0)
    ctx.kube.reconcile()
    asyncio.run(mon.reconcile_once())
    ctx.kube.delete_pytorchjob(ctx.namespace, jid)
    asyncio.run(mon.reconcile_once())  # first pass without it: within the grace period
    assert c.get(f"/api/v1/jobs/{jid}").json()["status"] != "failed"
    mon.orphan_grace_s = 0
    asyncio.run(mon.reconcile_once())
    j = c.get(f"/api/v1/jobs/{jid}").json()
    assert j["status"] == "failed" and j["metadata"]["reason"] == "PyTorchJobMissing"
    assert c.get(f"/api/v1/jobs/{keep}").json()["status"] != "failed"


def test_deleting_a_failed_job_removes_its_pytorchjob(env):
    """The monitor removes succeeded PyTorchJobs only; a failed one stays for inspection until the
    user deletes the job, which then takes the cluster object along."""
    ctx, c = env
    jid = submit(c)
    mon = JobMonitor(ctx, interval=0)
    for _ in range(40):  # every (re)start fails: backoffLimit restarts, then Failed
        ctx.kube.fail_next(jid)
        ctx.kube.reconcile()
        asyncio.run(mon.reconcile_once())
        if c.get(f"/api/v1/jobs/{jid}").json()["status"] == "failed":
            break
    assert c.get(f"/api/v1/jobs/{jid}").json()["status"] == "failed"
    assert jid in [j["metadata"]["name"] for j in ctx.kube.list_pytorchjobs(ctx.namespace)]
    r = c.request("DELETE", "/api/v1/jobs/delete", json={"job_ids": [jid]})
    assert r.status_code == 200 and ctx.kube.list_pytorchjobs(ctx.namespace) == []


def test_failed_job_insert_takes_the_pytorchjob_back(env, monkeypatch):
    """The PyTorchJob is created before the job document; when the insert fails the submission must
    not leave a job on the cluster that no DB record (and so no monitor pass) will ever claim."""
    ctx, c = env

    async def broken(**kw):
        raise RuntimeError("mongo write timeout")

    monkeypatch.setattr(ctx.store, "create_job", broken)
    r = c.post("/api/v1/jobs", data=FORM)
    assert r.status_code == 500 and "mongo write timeout" in r.json()["detail"]
    assert ctx.kube.list_pytorchjobs(ctx.namespace) == []


def test_rejected_submissions_leave_no_spooled_upload(env, monkeypatch, tmp_path):
    """Dataset files are spooled to disk while the form streams in; a submission refused after that
    (bad model, bad arguments, a form that breaks mid-upload) must not leave the file behind."""
    from finetune_controller_amd.controlplane.api import forms

    ctx, c = env
    spool = tmp_path / "spool"
    monkeypatch.setattr(forms, "UPLOAD_DIR", str(spool))

    def upload(**over):
        files = {"dataset": ("train.jsonl", io.BytesIO(b'{"text": "hi"}\n' * 1000), "application/json")}
        return c.post("/api/v1/jobs", data=dict(FORM, **over), files=files)

    assert upload(model="Nope").status_code == 404
    r = upload(arguments="[1, 2]")
    assert r.status_code == 400 and "expected an object" in r.json()["detail"]
    assert list(spool.iterdir()) == []
    # a field past the size bound AFTER the file part: the parser fails and removes what it spooled
    monkeypatch.setattr(forms, "MAX_FIELD_BYTES", 64)
    b = "ftcboundary"
    parts = [f'--{b}\r\nContent-Disposition: form-data; name="dataset"; filename="t.jsonl"\r\n'
             f"Content-Type: application/json\r\n\r\n{'x' * 5000}\r\n"]
    for k, v in dict(FORM, dataset_description="d" * 4096).items():
        parts.append(f'--{b}\r\nContent-Disposition: form-data; name="{k}"\r\n\r\n{v}\r\n')
    body = ("".join(parts) + f"--{b}--\r\n").encode()
    r = c.post("/api/v1/jobs", content=body, headers={"content-type": f"multipart/form-data; boundary={b}"})
    assert r.status_code == 422 and "too large" in r.json()["detail"]
    assert list(spool.iterdir()) == []
    monkeypatch.setattr(forms, "MAX_FIELD_BYTES", 1 << 20)
    # a body cut off inside the file part (no closing delimiter) is not a dataset
    fields = "".join(f'--{b}\r\nContent-Disposition: form-data; name="{k}"\r\n\r\n{v}\r\n' for k, v in FORM.items())
    cut = (fields + f'--{b}\r\nContent-Disposition: form-data; name="dataset"; filename="t.jsonl"\r\n\r\n'
           + '{"text": "hel').encode()
    r = c.post("/api/v1/jobs", content=cut, headers={"content-type": f"multipart/form-data; boundary={b}"})
    assert r.status_code == 422 and "truncated" in r.json()["detail"]
    assert list(spool.iterdir()) == [] and not ctx.kube.list_pytorchjobs(ctx.namespace)
    # an urlencoded form is bounded too (it cannot carry a file)
    monkeypatch.setattr(forms, "MAX_URLENCODED_BYTES", 1024)
    r = c.post("/api/v1/jobs", content=b"model_name=x&arguments=" + b"a" * 4096,
               headers={"content-type": "application/x-www-form-urlencoded"})
    assert r.status_code == 422 and "too large" in r.json()["detail"]


def test_dataset_upload_reuse_url_and_delete(env, monkeypatch):
    ctx, c = env
    files = {"dataset": ("train.jsonl", io.BytesIO(b'{"text": "hello"}\n' * 10), "application/json")}
    r = c.post("/api/v1/jobs", data=dict(FORM, dataset_description="tiny"), files=files)
    assert r.status_code == 200, r.text
    jid = r.json()["job_id"]
    job = ctx.kube.get_pytorchjob(ctx.namespace, jid)
    init = job["spec"]["pytorchReplicaSpecs"]["Master"]["template"]["spec"]["initContainers"]
    assert "dataset/train.jsonl" in init[0]["args"][0]
    all_ds = c.get("/api/v1/datasets/all").json()
    assert len(all_ds) == 1 and "s3_uri" not in all_ds[0]["dataset"] and all_ds[0]["dataset_name"] == "train.jsonl"
    ds_id = all_ds[0]["id"]
    jid2 = submit(c, dataset_id=ds_id)
    assert c.get(f"/api/v1/jobs/{jid2}").json()["dataset_id"] == ds_id
    assert c.post("/api/v1/jobs", data=dict(FORM, dataset_id="0" * 24)).status_code == 404

    def handler(req):
        return httpx.Response(200, content=b"a,b\n1,2\n", headers={"Content-Disposition": 'attachment; filename="x.csv"'})

    monkeypatch.setattr(services, "_http_client", lambda *a, **k: httpx.Client(transport=httpx.MockTransport(handler)))
    jid3 = submit(c, dataset_url="https://example.org/data/x.csv")
    page = c.get("/api/v1/datasets", params={"page_size": 10}).json()
    assert page["total"] == 2
    urls = [i for i in page["items"] if i["dataset_name"] == "x.csv"][0]
    assert urls["meta_"]["data"]["Source"] == "https://example.org/data/x.csv"
    first = [i for i in page["items"] if i["dataset_name"] == "train.jsonl"][0]
    assert first["job_ref_names"] == ["my run", "my run"]
    assert c.delete(f"/api/v1/datasets/{ds_id}").json() == {"message": "Dataset deleted successfully"}
    assert c.delete(f"/api/v1/datasets/{ds_id}").status_code == 404
    assert jid3


def test_promotion_state_changes_are_claimed_atomically(env):
    """Promote and unpromote claim the promotion state with one conditional update before their
    background copy / delete runs: a promote during an unpromotion (same prefix) is refused, and of two
    racing claims only one wins."""
    from finetune_controller_amd.controlplane.schemas.db import PromotionStatus as PS

    ctx, c = env
    jid = submit(c)
    settle(ctx)

    async def claims():
        dest = "s3://ftc-deploy/x/" + jid
        busy = [PS.IN_PROGRESS, PS.DELETING, PS.COMPLETED]
        first = await ctx.store.claim_job_promotion(jid, PS.IN_PROGRESS, dest, unless=busy)
        second = await ctx.store.claim_job_promotion(jid, PS.IN_PROGRESS, dest, unless=busy)
        await ctx.store.update_job_promotion(jid, PS.COMPLETED, dest)
        un1 = await ctx.store.claim_job_promotion(jid, PS.DELETING, dest, when=[PS.COMPLETED])
        un2 = await ctx.store.claim_job_promotion(jid, PS.DELETING, dest, when=[PS.COMPLETED])
        return first, second, un1, un2

    assert asyncio.run(claims()) == (True, False, True, False)
    # the job is now being unpromoted: a promote would copy into the prefix being deleted
    r = c.post(f"/api/v1/jobs/{jid}/promote")
    assert r.status_code == 409 and "unpromoted" in r.json()["detail"]
    assert c.get(f"/api/v1/jobs/{jid}").json()["promoted"] == "deleting"


def test_promote_unpromote_artifacts_delete(env):
    ctx, c = env
    jid = submit(c)
    r = c.post(f"/api/v1/jobs/{jid}/promote")
    assert r.status_code == 200 and r.json()["detail"] == "Cannot promote running job"  # reference quirk
    settle(ctx)
    r = c.post(f"/api/v1/jobs/{jid}/promote").json()
    assert r["status"] == "promotion_initiated"
    j = c.get(f"/api/v1/jobs/{jid}").json()
    assert j["promoted"] == "completed" and j["destination_uri"] == f"s3://ftc-deploy/language/llama3-8b/lora/{jid}"
    assert j["status_merged"] == "deployed"
    promoted = ctx.objects.list("ftc-deploy", f"language/llama3-8b/lora/{jid}")
    assert {o.Key.rsplit("/", 1)[1] for o in promoted} >= {"metrics.csv"}
    urls = c.get(f"/api/v1/admin/artifacts/presigned_urls/{jid}").json()["artifacts"]
    assert {u["key"] for u in urls} >= {"metrics.csv", "adapter_config.json"}
    z = c.get(f"/api/v1/admin/artifacts/{jid}")
    assert z.status_code == 200 and z.headers["content-type"] == "application/zip"
    assert "metrics.csv" in zipfile.ZipFile(io.BytesIO(z.content)).namelist()
    # rate limit: promote is 2/minute per client
    assert c.post(f"/api/v1/jobs/{jid}/unpromote").json()["status"] == "unpromotion_initiated"
    assert c.post(f"/api/v1/jobs/{jid}/promote").status_code == 429
    j = c.get(f"/api/v1/jobs/{jid}").json()
    assert j["promoted"] == "not_promoted" and not ctx.objects.list("ftc-deploy", "language/")
    r = c.request("DELETE", "/api/v1/jobs/delete", json={"job_ids": [jid]})
    assert r.json() == {"job_id": {"message": "Jobs deleted successfully"}}
    assert c.get(f"/api/v1/jobs/{jid}").status_code == 404
    assert not ctx.objects.list("ftc-bucket", f"finetune_jobs/default_user/{jid}")


def test_admin_poll_and_clean(env):
    ctx, c = env
    jid = submit(c)
    ctx.kube.reconcile()
    ctx.kube.reconcile()
    st = c.get(f"/api/v1/admin/job/poll/{jid}").json()["status"]
    assert st["type"] in ("Created", "Running") and "events" in st and "restart_count" in st
    assert c.get("/api/v1/admin/job/poll/nope").status_code == 404
    settle(ctx)
    jid2 = submit(c)  # still running -> skipped by clean
    r = c.delete("/api/v1/admin/jobs/default_user").json()
    assert r["jobs"] == [jid] and r["skipped"][0]["job_id"] == jid2


def test_websocket_log_stream(env):
    ctx, c = env
    jid = submit(c)
    settle(ctx, rounds=3)  # running, some log lines
    # pods of the succeeded job are deleted; stream a running job instead
    jid2 = submit(c)
    ctx.kube.reconcile()
    ctx.kube.reconcile()
    asyncio.run(JobMonitor(ctx, interval=0).reconcile_once())
    ctx.kube.reconcile()
    with c.websocket_connect(f"/api/v1/logs/{jid2}?follow=false&full_log=true") as ws:
        msgs = []
        try:
            while True:
                msgs.append(ws.receive_text())
        except Exception:
            pass
    text = "\n".join(msgs)
    assert "Fetching all previous logs" in text and "Epoch 0" in text
    assert "simulated training container" not in text  # suppressed until the first "Epoch" line
    assert jid


def test_dev_auth_routes(env):
    ctx, c = env
    tok = c.get("/auth/generate", params={"user": "erin"}).json()["token"]
    assert c.get("/auth/verify", params={"token": tok}).json()["sub"] == "erin"
    r = c.get("/auth/cookie", params={"user": "frank"})
    assert r.status_code == 200 and "bridge-user" in r.cookies
    schema = c.get("/openapi.json").json()
    assert schema["components"]["securitySchemes"]["BearerAuth"]["scheme"] == "bearer"
    assert schema["paths"]["/api/v1/jobs"]["post"]["security"] == [{"BearerAuth": []}]


def test_auth_enforced_ownership_and_model_scopes(tmp_path):
    ctx = AppContext.local(workdir=str(tmp_path), run_processes=False, ENVIRONMENT="local")
    app = create_app(ctx, run_monitor=False, force_auth=True,
                     validator_factory=lambda: type("V", (), {"validate_token": staticmethod(_reject)})())
    with TestClient(app) as c:
        from finetune_controller_amd.controlplane.auth.security import dev_generate_token

        a = dev_generate_token("dev-secret", "HS256", "alice", ["Llama3-8B"])
        b = dev_generate_token("dev-secret", "HS256", "bob", ["GPT2-small"])
        assert c.get("/api/v1/models").status_code == 401
        ha, hb = {"Authorization": f"Bearer {a}"}, {"Authorization": f"Bearer {b}"}
        assert list(c.get("/api/v1/models", headers=hb).json()) == ["GPT2-small-FT"]
        assert c.post("/api/v1/jobs", data=FORM, headers=hb).status_code == 404  # model not in bob's scopes
        jid = c.post("/api/v1/jobs", data=dict(FORM, user_id="ignored"), headers=ha).json()["job_id"]
        assert c.get(f"/api/v1/jobs/{jid}", headers=ha).json()["user_id"] == "alice"
        assert c.get(f"/api/v1/jobs/{jid}", headers=hb).status_code == 400
        assert c.get("/api/v1/jobs", headers=hb).json()["total"] == 0
        with pytest.raises(Exception):
            with c.websocket_connect(f"/api/v1/logs/{jid}") as ws:  # no credentials
                ws.receive_text()


async def _reject(token):
    raise RuntimeError("IdP unavailable")


class _StubValidator:
    """Accepts any token and reports its (unverified) subject -- the auth middleware's contract."""

    async def validate_token(self, token):
        from finetune_controller_amd.controlplane.auth import jwt as jose

        return {"active": True, "sub": jose.get_unverified_claims(token)["sub"]}


def test_admin_routes_require_admin_or_owner(tmp_path):
    """With auth on: user B cannot wipe user A's jobs (403), list cluster jobs or poll A's job; A may
    clean and poll their own; a token carrying the admin scope may do everything."""
    from finetune_controller_amd.controlplane.auth.security import dev_generate_token

    ctx = AppContext.local(workdir=str(tmp_path), run_processes=False)
    ctx.settings.ADMIN_USERS = ["root_admin"]
    app = create_app(ctx, run_monitor=False, force_auth=True, validator_factory=_StubValidator)
    models = ctx.registry.all_inference_names() + list(ctx.registry.names())
    tok = {u: dev_generate_token("k", "HS256", u, models) for u in ("alice", "bob", "root_admin")}
    tok["scoped"] = dev_generate_token("k", "HS256", "carol", models + [ctx.settings.ADMIN_SCOPE])

    def h(u):
        return {"Authorization": f"Bearer {tok[u]}"}

    with TestClient(app) as c:
        r = c.post("/api/v1/jobs", data=FORM, headers=h("alice"))
        assert r.status_code == 200, r.text
        jid = r.json()["job_id"]
        ctx.kube.reconcile()
        ctx.kube.reconcile()
        assert c.delete("/api/v1/admin/jobs/alice", headers=h("bob")).status_code == 403
        assert c.get("/api/v1/admin/jobs/list", headers=h("bob")).status_code == 403
        assert c.get(f"/api/v1/admin/job/poll/{jid}", headers=h("bob")).status_code == 403
        assert c.get(f"/api/v1/admin/job/poll/{jid}", headers=h("alice")).status_code == 200
        assert c.get("/api/v1/admin/jobs/list", headers=h("root_admin")).json()["jobs"] == [jid]
        assert c.get("/api/v1/admin/jobs/list", headers=h("scoped")).status_code == 200
        # the job still runs: the owner's clean skips it but is allowed
        r = c.delete("/api/v1/admin/jobs/alice", headers=h("alice"))
        assert r.status_code == 200 and r.json()["skipped"][0]["job_id"] == jid
        assert c.get(f"/api/v1/jobs/{jid}", headers=h("alice")).status_code == 200
