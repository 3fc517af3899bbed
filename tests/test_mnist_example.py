"""The reference's example job (MNIST) on this framework's worker: the example's command line, IDX /
npz / synthetic data, single-process and 2-rank gloo DDP training, and the job through the API on a
FakeCluster CPU worker."""
import asyncio
import gzip
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import pytest
import torch

from finetune_controller_amd.train import mnist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _write_idx(path, arr: np.ndarray):
    hdr = bytes([0, 0, 0x08, arr.ndim]) + b"".join(int(d).to_bytes(4, "big") for d in arr.shape)
    op = gzip.open if path.endswith(".gz") else open
    with op(path, "wb") as f:
        f.write(hdr + arr.astype(np.uint8).tobytes())


def test_idx_and_npz_loaders(tmp_path):
    x, y = mnist.synthetic_mnist(50, 0)
    d = tmp_path / "idx"
    d.mkdir()
    _write_idx(str(d / "train-images-idx3-ubyte.gz"), x)
    _write_idx(str(d / "train-labels-idx1-ubyte.gz"), y)
    _write_idx(str(d / "t10k-images-idx3-ubyte"), x[:10])
    _write_idx(str(d / "t10k-labels-idx1-ubyte"), y[:10])
    xtr, ytr, xte, yte, src = mnist.load_mnist(str(d), 0, 0, 0)
    assert src == "idx" and np.array_equal(xtr, x) and np.array_equal(ytr, y) and xte.shape == (10, 28, 28)
    d2 = tmp_path / "npz"
    d2.mkdir()
    np.savez(d2 / "mnist.npz", x_train=x, y_train=y, x_test=x[:5], y_test=y[:5])
    assert mnist.load_mnist(str(d2), 0, 0, 0)[4] == "npz"
    assert mnist.load_mnist(str(tmp_path / "none"), 20, 10, 0)[4] == "synthetic"


def test_mnist_example_trains_and_saves(tmp_path):
    last = mnist.run(mnist.build_parser().parse_args(
        ["--epochs", "2", "--train-size", "3000", "--test-size", "500", "--no-cuda", "--log-interval", "20",
         "--save-model", "--dataset_path", str(tmp_path / "none"), "--checkpoint_path", str(tmp_path / "out")]))
    assert last["epoch"] == 2 and last["accuracy"] > 90.0 and last["lr"] == pytest.approx(0.7)
    rows = open(tmp_path / "out" / "metrics.csv").read().splitlines()
    assert rows[0].startswith("epoch,step,loss,lr,test_loss,accuracy") and len(rows) > 4
    sd = torch.load(tmp_path / "out" / "mnist_cnn.pt", weights_only=True)
    assert sd["fc2.weight"].shape == (10, 128)


def test_mnist_example_two_rank_gloo(tmp_path):
    env = dict(os.environ, PYTHONPATH=REPO, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), "-m", "finetune_controller_amd.train.mnist",
           "--epochs", "1", "--train-size", "2001", "--test-size", "300", "--no-cuda", "--log-interval", "10",
           "--dataset_path", str(tmp_path / "none"), "--checkpoint_path", str(tmp_path / "out")]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "world=2" in r.stdout and "Train Epoch: 1" in r.stdout and "Training complete" in r.stdout


def _wait_for(pred, timeout=240.0):
    t0 = time.time()
    while time.time() - t0 < timeout:
        if pred():
            return
        time.sleep(1.5)  # under the 50/min rate limit of GET /api/v1/jobs/{id}
    raise TimeoutError("condition not reached")


def test_mnist_job_through_api_on_fakecluster(tmp_path):
    from fastapi.testclient import TestClient

    from finetune_controller_amd.controlplane.api.app import create_app
    from finetune_controller_amd.controlplane.context import AppContext
    from finetune_controller_amd.controlplane.monitor.reconciler import JobMonitor
    from finetune_controller_amd.controlplane.spec.models.builtin import MNIST_MI355X

    class MNISTSmall(MNIST_MI355X):
        name: str = "MNIST-small"
        command: list[str] = ["/bin/bash", "-c", "python -m finetune_controller_amd.train.mnist --train-size=1500 "
                                                 "--test-size=300"]

    cmd = MNIST_MI355X().run_cmd()[-1]
    assert cmd.startswith("python -m finetune_controller_amd.train.mnist --batch-size=64 --test-batch-size=1000")
    assert "torchrun --standalone --nproc-per-node=4" in MNIST_MI355X(accelerator_count=4).run_cmd()[-1]
    ctx = AppContext.local(workdir=str(tmp_path), run_processes="cpu")
    ctx.registry.register(MNISTSmall)
    ctx.kube.sync_interval = 0.2
    app = create_app(ctx, run_monitor=False, force_auth=False)
    with TestClient(app) as c:
        r = c.post("/api/v1/jobs", data={"job_name": "mnist e2e", "model": "MNIST-small", "device": "cpu",
                                        "task": "classification",
                                        "arguments": json.dumps({"epochs": 1, "no_cuda": True, "save_model": True})})
        assert r.status_code == 200, r.text
        jid = r.json()["job_id"]
        ctx.kube.start(tick=0.1)
        try:
            def done():
                asyncio.run(JobMonitor(ctx, interval=0).reconcile_once())
                r = c.get(f"/api/v1/jobs/{jid}")
                assert r.status_code == 200, r.text
                return r.json()["status"] in ("completed", "failed")

            _wait_for(done)
        finally:
            ctx.kube.stop()
        pod_logs = "\n".join("\n".join(p.logs) for p in ctx.kube.pods.values()) + \
            "\n".join("\n".join(v) for v in ctx.kube.deleted_pod_logs.values())
        assert c.get(f"/api/v1/jobs/{jid}").json()["status"] == "completed", pod_logs[-3000:]
        assert "Train Epoch: 1" in pod_logs
        m = c.get(f"/api/v1/jobs/{jid}/metrics").json()
        assert any(row.get("accuracy") for row in m["metrics"])
        keys = {u["key"] for u in c.get(f"/api/v1/admin/artifacts/presigned_urls/{jid}").json()["artifacts"]}
        assert {"metrics.csv", "mnist_cnn.pt"} <= keys
