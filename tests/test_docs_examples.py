"""docs/models.md stays true: the walkthrough specs in docs/examples/custom_models load through the
registry's custom-directory loader, self-check, submit through the API on the FakeCluster with the
documented manifests, and the walkthrough's training script honours the worker contract."""
import csv
import json
import os
import subprocess
import sys

import numpy as np
from fastapi.testclient import TestClient

from finetune_controller_amd.controlplane.api.app import create_app
from finetune_controller_amd.controlplane.context import AppContext

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EX = os.path.join(ROOT, "docs", "examples")


def _csv(path, n=64, seed=0):
    rng = np.random.default_rng(seed)
    x = rng.normal(size=(n, 3))
    y = x @ np.array([1.5, -2.0, 0.5]) + 0.3
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["logp", "tpsa", "mw", "solubility"])
        for xi, yi in zip(x, y):
            w.writerow([*(f"{v:.5f}" for v in xi), f"{yi:.5f}"])


def test_example_specs_self_check():
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    for f in ("solubility_regressor.py", "llama3_8b_lora_r64.py"):
        r = subprocess.run([sys.executable, os.path.join(EX, "custom_models", f)], env=env, capture_output=True,
                           text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        assert "--checkpoint_path=/data/artifacts" in r.stdout


def test_walkthrough_specs_through_the_api(tmp_path):
    ctx = AppContext.local(workdir=str(tmp_path), run_processes=False)
    assert ctx.registry.load_custom(os.path.join(EX, "custom_models")) == 2
    app = create_app(ctx, run_monitor=False, force_auth=False)
    ds = tmp_path / "descriptors.csv"
    _csv(ds)
    with TestClient(app) as c:
        models = c.get("/api/v1/models").json()
        assert set(models["Solubility-Regressor"]["arguments"]) == {"epochs", "lr", "l2", "target_column"}
        # dataset_required: refused without a dataset
        r = c.post("/api/v1/jobs", data={"job_name": "nods", "model": "Solubility-Regressor", "device": "cpu",
                                        "task": "regression", "user_id": "alice"})
        assert r.status_code == 400 and "dataset is required" in r.text
        # constraint violations name the field
        r = c.post("/api/v1/jobs", data={"job_name": "bad", "model": "Solubility-Regressor", "device": "cpu",
                                        "task": "regression", "user_id": "alice", "arguments": '{"epochs": 0}'},
                   files={"dataset": ("d.csv", ds.read_bytes(), "text/csv")})
        assert r.status_code == 400 and "epochs" in r.text
        r = c.post("/api/v1/jobs", data={"job_name": "sol-v1", "model": "Solubility-Regressor", "device": "cpu",
                                        "task": "regression", "user_id": "alice", "arguments": '{"epochs": 7}'},
                   files={"dataset": ("d.csv", ds.read_bytes(), "text/csv")})
        assert r.status_code == 200, r.text
        job = ctx.kube.objects[("kubeflow.org", "pytorchjobs", ctx.namespace, r.json()["job_id"])]
        pod = job["spec"]["pytorchReplicaSpecs"]["Master"]["template"]["spec"]
        main = pod["containers"][0]
        assert main["name"] == "pytorch" and main["image"].endswith("solubility-trainer:0.1")
        assert "python /app/train_regressor.py --epochs=7" in main["command"][-1]
        assert "touch /data/artifacts/done.txt" in main["command"][-1]  # success sentinel (failed.txt otherwise)
        assert "amd.com/gpu" not in main["resources"].get("requests", {})
        assert main["resources"]["requests"]["cpu"] == 2
        assert pod["initContainers"][0]["name"] == "dataset-downloader"
        # walkthrough B: 2-GPU LoRA variant
        r = c.post("/api/v1/jobs", data={"job_name": "r64", "model": "Llama3-8B-LoRA-r64-8k", "device": "mi355x",
                                        "task": "causal_lm", "user_id": "alice", "arguments": '{"max_steps": 50}'})
        assert r.status_code == 200, r.text
        job = ctx.kube.objects[("kubeflow.org", "pytorchjobs", ctx.namespace, r.json()["job_id"])]
        main = job["spec"]["pytorchReplicaSpecs"]["Master"]["template"]["spec"]["containers"][0]
        cmd = main["command"][-1]
        assert "torchrun --standalone --nproc-per-node=2" in cmd
        assert "--lora-r=64" in cmd and "--seq-len=8192" in cmd and "--max-steps=50" in cmd
        assert main["resources"]["limits"]["amd.com/gpu"] == 2


def test_walkthrough_training_script_contract(tmp_path):
    ds, out = tmp_path / "dataset", tmp_path / "artifacts"
    ds.mkdir()
    _csv(ds / "descriptors.csv", n=200)
    r = subprocess.run([sys.executable, os.path.join(EX, "train_regressor.py"), "--epochs=30", "--lr=0.1",
                        f"--dataset_path={ds}", f"--checkpoint_path={out}"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.splitlines()[0].startswith("Epoch 0")
    rows = list(csv.DictReader(open(out / "metrics.csv")))
    assert len(rows) == 30 and float(rows[-1]["loss"]) < 0.05 * float(rows[0]["loss"])
    model = json.load(open(out / "model.json"))
    assert model["columns"] == ["logp", "tpsa", "mw"]
