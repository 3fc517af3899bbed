"""The minimum end-to-end slice on an MI355X: a LoRA job submitted through
``POST /api/v1/jobs``, admitted by the emulated Kueue with an ``amd.com/gpu`` request, executed for
real by the FakeCluster as a subprocess of this repository's trainer ON THE GPU (HIP kernels), its
artifacts synced, its metrics ingested by the monitor, PEFT adapter files downloadable."""
import json
import os
from typing import ClassVar

import pytest
from fastapi.testclient import TestClient

from finetune_controller_amd.controlplane.api.app import create_app
from finetune_controller_amd.controlplane.context import AppContext
from finetune_controller_amd.controlplane.spec.models.builtin import Llama3_8B_LoRA, LoRAArguments

pytestmark = pytest.mark.gpu


class LlamaSmokeLoRA(Llama3_8B_LoRA):
    """The Llama-3 attention geometry at toy width (preset llama-smoke), one MI355X."""

    name: str = "Llama-smoke-LoRA"
    inference_name: str | None = "Llama-smoke"
    training_arguments: LoRAArguments = LoRAArguments(batch_size=2, seq_len=256, max_steps=6, log_interval=2,
                                                      warmup_steps=1, lr=1e-3)
    model_preset: ClassVar[str] = "llama-smoke"


def test_lora_job_runs_on_the_gpu_through_the_api(tmp_path):
    from test_e2e_fakecluster import run_monitor, wait_for

    ctx = AppContext.local(workdir=str(tmp_path), run_processes=True)
    ctx.registry.register(LlamaSmokeLoRA)
    ctx.kube.sync_interval = 0.2
    app = create_app(ctx, run_monitor=False, force_auth=False)
    with TestClient(app) as c:
        text = ("the quick brown fox jumps over the lazy dog. " * 400).encode()
        r = c.post("/api/v1/jobs", data={"job_name": "gpu e2e", "model": "Llama-smoke-LoRA", "device": "mi355x",
                                        "task": "causal_lm", "user_id": "alice"},
                   files={"dataset": ("corpus.txt", text, "text/plain")})
        assert r.status_code == 200, r.text
        jid = r.json()["job_id"]
        job = ctx.kube.objects[("kubeflow.org", "pytorchjobs", ctx.namespace, jid)]
        cont = job["spec"]["pytorchReplicaSpecs"]["Master"]["template"]["spec"]["containers"][0]
        assert cont["resources"]["limits"]["amd.com/gpu"] == 1
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
        assert len(m) >= 2 and all(row["tokens_per_sec"] > 0 for row in m)
        urls = {u["key"]: u["url"] for u in c.get(f"/api/v1/admin/artifacts/presigned_urls/{jid}").json()["artifacts"]}
        assert {"adapter_model.safetensors", "adapter_config.json", "metrics.csv", "training_config.json"} <= set(urls)
        # the worker really ran the HIP path on the GPU
        art = os.path.join(str(tmp_path), "s3", ctx.settings.S3_BUCKET_NAME)
        cfgs = [os.path.join(d, f) for d, _, fs in os.walk(art) for f in fs if f == "training_config.json"]
        runtime = json.load(open(cfgs[0]))["runtime"]
        assert runtime["kernels"] == "hip" and runtime["device"].startswith("cuda"), runtime
