"""End-to-end on the FakeCluster (SURVEY.md §4 "[new] Cluster simulation"):

* BASELINE.json config #1 -- a GPT-2 full fine-tune PyTorchJob submitted through the REST API, admitted
  by (emulated) Kueue on the CPU worker, executed for real as a subprocess running this repository's
  trainer, artifacts synced by the emulated sidecar, state + metrics reconciled by the monitor;
* BASELINE.json config #5 -- Kueue multi-tenant: 4 concurrent Llama-3-8B LoRA jobs @ 2 GPUs under an
  ``amd.com/gpu: 8`` ClusterQueue, the 5th waits with a queue position and is admitted when quota frees;
* failure detection / restart path with fault injection (``backoffLimit`` retries, then Failed).
"""
import asyncio
import json
import os
import time

import pytest
from fastapi.testclient import TestClient
from pydantic import Field

from finetune_controller_amd.controlplane.api.app import create_app
from finetune_controller_amd.controlplane.context import AppContext
from finetune_controller_amd.controlplane.monitor.reconciler import JobMonitor
from finetune_controller_amd.controlplane.spec.models.builtin import GPT2SmallFT, LMTrainingArguments
from typing import ClassVar


class GPT2TinyFT(GPT2SmallFT):
    """Same spec as GPT2-small-FT with the test-sized GPT-2 family member."""

    name: str = "GPT2-tiny-FT"
    inference_name: str | None = "GPT2-tiny"
    model_preset: ClassVar[str] = "gpt2-tiny"
    training_arguments: LMTrainingArguments = LMTrainingArguments(batch_size=2, seq_len=64, lr=1e-3, max_steps=6,
                                                                  log_interval=2, warmup_steps=1)


def wait_for(pred, timeout=120.0, step=0.2):
    t0 = time.time()
    while time.time() - t0 < timeout:
        v = pred()
        if v:
            return v
        time.sleep(step)
    raise TimeoutError("condition not reached")


def run_monitor(ctx):
    asyncio.run(JobMonitor(ctx, interval=0).reconcile_once())


@pytest.mark.parametrize("model", ["GPT2-tiny-FT", pytest.param("GPT2-small-FT", marks=pytest.mark.slow)])
def test_gpt2_full_ft_job_runs_on_cpu_worker(tmp_path, model):
    ctx = AppContext.local(workdir=str(tmp_path), run_processes="cpu")
    ctx.registry.register(GPT2TinyFT)
    ctx.kube.sync_interval = 0.2
    app = create_app(ctx, run_monitor=False, force_auth=False)
    args = {"max_steps": 2, "seq_len": 64, "batch_size": 1, "log_interval": 1} if model == "GPT2-small-FT" else {}
    with TestClient(app) as c:
        files = {"dataset": ("corpus.txt", ("the quick brown fox jumps over the lazy dog\n" * 200).encode(), "text/plain")}
        r = c.post("/api/v1/jobs", data={"job_name": "gpt2 e2e", "model": model, "device": "cpu",
                                        "task": "causal_lm", "arguments": json.dumps(args)}, files=files)
        assert r.status_code == 200, r.text
        jid = r.json()["job_id"]
        ctx.kube.start(tick=0.1)
        try:
            def done():
                run_monitor(ctx)
                r = c.get(f"/api/v1/jobs/{jid}")
                assert r.status_code == 200, r.text
                return r.json()["status"] in ("completed", "failed")

            # the GET route is rate-limited to 50/min per client (reference app/main.py), so poll
            # below that rate: a slow CPU worker would otherwise see 429s.
            wait_for(done, timeout=240, step=1.5)
        finally:
            ctx.kube.stop()
        j = c.get(f"/api/v1/jobs/{jid}").json()
        pod_logs = "\n".join("\n".join(p.logs) for p in ctx.kube.pods.values()) + \
            "\n".join("\n".join(v) for v in ctx.kube.deleted_pod_logs.values())
        assert j["status"] == "completed", pod_logs[-3000:]
        assert ("gpt2 e2e", "Succeeded") not in ctx.kube.history  # history keyed by job id
        assert (jid, "Suspended") in ctx.kube.history and (jid, "Running") in ctx.kube.history
        assert "[dataset-downloader] download" in pod_logs and "Epoch 0" in pod_logs
        m = c.get(f"/api/v1/jobs/{jid}/metrics").json()
        assert len(m["metrics"]) >= 2 and {"loss", "tokens_per_sec", "step"} <= set(m["metrics"][0])
        keys = {u["key"] for u in c.get(f"/api/v1/admin/artifacts/presigned_urls/{jid}").json()["artifacts"]}
        assert {"metrics.csv", "config.json", "training_config.json", "model.safetensors.index.json"} <= keys
        assert "done.txt" not in keys


def test_kueue_multi_tenant_gpu_quota(tmp_path):
    ctx = AppContext.local(workdir=str(tmp_path), run_processes=False)
    ctx.kube.sim_ticks = 50  # keep the admitted jobs running
    app = create_app(ctx, run_monitor=False, force_auth=False)
    with TestClient(app) as c:
        ids = []
        for i in range(5):
            r = c.post("/api/v1/jobs", data={"job_name": f"tenant{i}", "model": "Llama3-8B-LoRA-2GPU",
                                            "device": "mi355x", "task": "causal_lm", "user_id": f"user{i}"})
            assert r.status_code == 200, r.text
            ids.append(r.json()["job_id"])
        # the 2-GPU spec alone yields the 2-GPU request and the 2-rank launch (no manifest edits)
        for jid in ids:
            job = ctx.kube.objects[("kubeflow.org", "pytorchjobs", ctx.namespace, jid)]
            cont = job["spec"]["pytorchReplicaSpecs"]["Master"]["template"]["spec"]["containers"][0]
            assert cont["resources"]["requests"]["amd.com/gpu"] == 2 and cont["resources"]["limits"]["amd.com/gpu"] == 2
            assert "--nproc-per-node=2" in cont["command"][-1]
        for _ in range(4):
            ctx.kube.reconcile()
        run_monitor(ctx)
        st = {jid: c.get(f"/api/v1/jobs/{jid}", params={}).json() for jid in ids}
        running = [j for j in ids if st[j]["status"] in ("starting", "running")]
        assert len(running) == 4, {j: st[j]["status"] for j in ids}
        assert st[ids[4]]["status"] == "queued" and st[ids[4]]["metadata"]["queue_pos"] == 1
        assert ctx.kube.usage["cluster-queue"]["amd.com/gpu"] == 8
        # finish one job -> quota frees -> the 5th is admitted
        c.post(f"/api/v1/jobs/{ids[0]}/cancel")
        for _ in range(3):
            ctx.kube.reconcile()
        run_monitor(ctx)
        assert c.get(f"/api/v1/jobs/{ids[4]}").json()["status"] in ("starting", "running")
        assert c.get(f"/api/v1/jobs/{ids[0]}").json()["status"] == "canceled"


def test_failure_restart_then_failed(tmp_path):
    ctx = AppContext.local(workdir=str(tmp_path), run_processes=False)
    ctx.kube.sim_ticks = 100
    app = create_app(ctx, run_monitor=False, force_auth=False)
    with TestClient(app) as c:
        jid = c.post("/api/v1/jobs", data={"job_name": "f", "model": "Llama3-8B-LoRA", "device": "mi355x",
                                          "task": "causal_lm"}).json()["job_id"]
        for _ in range(3):
            ctx.kube.reconcile()
        run_monitor(ctx)
        assert c.get(f"/api/v1/jobs/{jid}").json()["status"] == "running"
        ctx.kube.kill_pod(ctx.namespace, jid, exit_code=137)  # OOM-kill the master
        ctx.kube.reconcile()
        ctx.kube.reconcile()
        run_monitor(ctx)
        seen = [t for j, t in ctx.kube.history if j == jid]
        assert "Restarting" in seen
        for _ in range(2):  # exhaust backoffLimit=2
            ctx.kube.kill_pod(ctx.namespace, jid)
            ctx.kube.reconcile()
            ctx.kube.reconcile()
        ctx.kube.kill_pod(ctx.namespace, jid)
        for _ in range(3):
            ctx.kube.reconcile()
        run_monitor(ctx)
        j = c.get(f"/api/v1/jobs/{jid}").json()
        assert j["status"] == "failed" and "exited with code" in j["metadata"]["message"]
        run_monitor(ctx)  # stopped jobs are not re-processed (fixed comparison)
        assert c.get(f"/api/v1/jobs/{jid}").json()["updated_at"] == j["updated_at"]
        poll = c.get(f"/api/v1/admin/job/poll/{jid}").json()["status"]
        assert poll["type"] == "Failed" and poll["restart_count"] >= 2


def test_mixed_pool_kueue_example_through_the_api(tmp_path):
    """deploy/kueue/examples (cohort "finetune": adapters + ddp ClusterQueues, cpu / mi355x-pool /
    mi355x-node flavors) with its device catalogue: 2-GPU LoRA jobs share the 8-GPU adapters pool,
    8-GPU full fine-tunes take whole nodes from the ddp queue, and each queue admits and queues
    independently."""
    import yaml

    from finetune_controller_amd.controlplane.k8s.fake import kueue_quotas_from_manifests

    ex = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "deploy", "kueue", "examples")
    docs = []
    for f in ("flavors.yaml", "cluster-queues.yaml", "local-queues.yaml"):
        docs += list(yaml.safe_load_all(open(os.path.join(ex, f))))
    flavors = {d["metadata"]["name"] for d in docs if d["kind"] == "ResourceFlavor"}
    for d in docs:
        if d["kind"] == "ClusterQueue":
            assert d["spec"]["cohort"] == "finetune"
            assert {f["name"] for g in d["spec"]["resourceGroups"] for f in g["flavors"]} <= flavors
    cqs, lqs = kueue_quotas_from_manifests(docs)
    assert cqs["adapters"]["amd.com/gpu"] == 8 and cqs["ddp"]["amd.com/gpu"] == 16
    ctx = AppContext.local(workdir=str(tmp_path), run_processes=False,
                           config_json=open(os.path.join(ex, "config.mixed.json")).read())
    ctx.kube.set_kueue(cqs, lqs)
    assert {ctx.devices.get_worker(n).local_queue for n in ctx.devices.list_workers()} <= set(lqs)
    ctx.kube.sim_ticks = 50
    app = create_app(ctx, run_monitor=False, force_auth=False)
    with TestClient(app) as c:
        def submit(model, device, i):
            r = c.post("/api/v1/jobs", data={"job_name": f"j{i}", "model": model, "device": device,
                                            "task": "causal_lm", "user_id": f"user{i}"})
            assert r.status_code == 200, r.text
            return r.json()["job_id"]

        lora = [submit("Llama3-8B-LoRA-2GPU", "mi355x", i) for i in range(5)]
        full = [submit("Llama3-8B-Full", "mi355x-node", 10 + i) for i in range(3)]
        for _ in range(4):
            ctx.kube.reconcile()
        run_monitor(ctx)
        st = {j: c.get(f"/api/v1/jobs/{j}").json()["status"] for j in lora + full}
        assert all(st[j] in ("starting", "running") for j in lora[:4])
        assert st[lora[4]] == "queued"
        assert all(st[j] in ("starting", "running") for j in full[:2]) and st[full[2]] == "queued"
        assert ctx.kube.usage["adapters"]["amd.com/gpu"] == 8 and ctx.kube.usage["ddp"]["amd.com/gpu"] == 16
        job = ctx.kube.objects[("kubeflow.org", "pytorchjobs", ctx.namespace, full[0])]
        assert job["metadata"]["labels"]["kueue.x-k8s.io/queue-name"] == "finetune-ddp-queue"


class GPT2TinyFT2Node(GPT2TinyFT):
    """Two replicas (Master + 1 Worker): the operator-injected PET_* rendezvous, torchrun per pod."""

    name: str = "GPT2-tiny-FT-2node"
    cluster_nodes: int = Field(default=2, ge=1, description="Total number of workers for training")


@pytest.mark.slow
def test_multi_node_job_trains_data_parallel_across_pods(tmp_path):
    """cluster_nodes=2 through the API: the FakeCluster starts Master and Worker pods with the
    training-operator's PET_NNODES / PET_NODE_RANK / PET_MASTER_* env, each pod's torchrun joins one
    2-rank gloo group, and the job completes with metrics reporting world size 2."""
    ctx = AppContext.local(workdir=str(tmp_path), run_processes="cpu")
    ctx.registry.register(GPT2TinyFT2Node)
    ctx.kube.sync_interval = 0.2
    app = create_app(ctx, run_monitor=False, force_auth=False)
    with TestClient(app) as c:
        files = {"dataset": ("corpus.txt", ("pack my box with five dozen liquor jugs\n" * 300).encode(), "text/plain")}
        r = c.post("/api/v1/jobs", data={"job_name": "2node", "model": "GPT2-tiny-FT-2node", "device": "cpu",
                                        "task": "causal_lm"}, files=files)
        assert r.status_code == 200, r.text
        jid = r.json()["job_id"]
        job = ctx.kube.objects[("kubeflow.org", "pytorchjobs", ctx.namespace, jid)]
        assert job["spec"]["pytorchReplicaSpecs"]["Worker"]["replicas"] == 1
        cmd = job["spec"]["pytorchReplicaSpecs"]["Master"]["template"]["spec"]["containers"][0]["command"][-1]
        assert "--nnodes=${PET_NNODES:-1}" in cmd and "--node-rank=${PET_NODE_RANK:-0}" in cmd
        ctx.kube.start(tick=0.1)
        try:
            def done():
                run_monitor(ctx)
                return c.get(f"/api/v1/jobs/{jid}").json()["status"] in ("completed", "failed")

            wait_for(done, timeout=300, step=1.5)
        finally:
            ctx.kube.stop()
        logs = "\n".join("\n".join(p.logs) for p in ctx.kube.pods.values()) + \
            "\n".join("\n".join(v) for v in ctx.kube.deleted_pod_logs.values())
        assert c.get(f"/api/v1/jobs/{jid}").json()["status"] == "completed", logs[-3000:]
        m = c.get(f"/api/v1/jobs/{jid}/metrics").json()["metrics"]
        assert m and all(int(row["world_size"]) == 2 for row in m), m[:2]
