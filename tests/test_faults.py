"""Failure detection and fault injection: the worker's fault hooks and detectors
(``utils.faults``), the rank-consistent resume they rely on, and the whole restart path on the
FakeCluster -- a lost peer (the RCCL-timeout case) in a 2-pod job ends in a completed job that resumed
from its checkpoint."""
import os
import subprocess
import sys
import threading
import time

import pytest
import torch

from finetune_controller_amd.parallel import dist as pdist
from finetune_controller_amd.train.trainer import TrainConfig, Trainer
from finetune_controller_amd.utils.faults import WATCHDOG_EXIT, FaultInjector, FaultSpec, StepWatchdog

from test_distributed import _hold, _rank_env, _run_ranks

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_fault_spec_parse():
    assert FaultSpec.parse("") is None and FaultSpec.parse(None) is None
    assert FaultSpec.parse("hang@3:rank=1") == FaultSpec("hang", 3, 1)
    assert FaultSpec.parse("oom@0") == FaultSpec("oom", 0, 0)
    for bad in ("explode@1", "crash", "crash@x", "crash@1:rank="):
        with pytest.raises(ValueError):
            FaultSpec.parse(bad)


def test_injector_fires_once_per_job_on_its_rank(tmp_path):
    spec = FaultSpec("crash", 2, rank=1)
    assert not FaultInjector(spec, rank=0, state_dir=str(tmp_path)).armed  # another rank's fault
    inj = FaultInjector(spec, rank=1, state_dir=str(tmp_path))
    inj.maybe_fire(0)
    inj.maybe_fire(1)
    with pytest.raises(RuntimeError, match="injected crash at step 2 on rank 1"):
        inj.maybe_fire(2)
    assert os.path.exists(tmp_path / spec.marker)
    # the restarted worker (a fresh injector over the same checkpoint dir) runs through
    again = FaultInjector(spec, rank=1, state_dir=str(tmp_path))
    assert not again.armed
    again.maybe_fire(2)


def test_oom_fault_is_a_sigkill(tmp_path):
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from finetune_controller_amd.utils.faults import FaultInjector, FaultSpec\n"
            "FaultInjector(FaultSpec.parse('oom@1'), 0, %r).maybe_fire(1)\n") % (ROOT, str(tmp_path))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert r.returncode == -9, r.stderr  # SIGKILL: the pod reports 137, like the kernel OOM killer
    assert "injected oom at step 1" in r.stderr


def test_step_watchdog_exits_124_with_stacks(capfd):
    fired = threading.Event()
    codes = []

    def exit_fn(code):
        codes.append(code)
        fired.set()

    wd = StepWatchdog(1.0, rank=3, exit_fn=exit_fn, poll_s=0.02)
    for i in range(10):  # beating keeps it quiet
        time.sleep(0.05)
        wd.beat(f"step {i}")
    assert not fired.is_set()
    assert fired.wait(5.0)
    wd.close()
    assert codes == [WATCHDOG_EXIT]
    err = capfd.readouterr().err
    assert "[watchdog] rank 3: no progress" in err and "last: step 9" in err
    assert "Thread" in err or "File" in err  # faulthandler's stack dump
    assert StepWatchdog(0)._thread is None  # 0 = disabled


def test_step_watchdog_first_step_grace():
    codes = []
    wd = StepWatchdog(0.1, exit_fn=codes.append, poll_s=0.02, first_timeout_s=3.0)
    time.sleep(0.3)  # a slow first step (warm-up): past timeout_s, inside the first-step limit
    assert codes == []
    wd.beat("step 1")
    time.sleep(0.6)  # from now on the plain limit applies
    wd.close()
    assert codes and codes[0] == WATCHDOG_EXIT


def test_step_watchdog_phase_limit():
    """A phase (the final save + closing barrier) gets its own limit: longer than a step's, still an exit
    when the phase never ends (a peer died in the barrier)."""
    codes = []
    wd = StepWatchdog(0.1, exit_fn=codes.append, poll_s=0.02, first_timeout_s=3.0)
    wd.beat("step 1")
    wd.phase("final save", 0.8)
    time.sleep(0.4)  # past the step limit, inside the phase limit
    assert codes == []
    time.sleep(0.8)
    wd.close()
    assert codes and codes[0] == WATCHDOG_EXIT


def test_slow_final_save_does_not_trip_the_watchdog(tmp_path, monkeypatch):
    """The watchdog covers steps, evaluations and checkpoints; the final artifact save (minutes for a
    full-FT model on rank 0, with the other ranks waiting in the barrier) runs under the save phase's
    longer limit."""
    from finetune_controller_amd.train import trainer as trmod

    codes = []
    real = trmod.StepWatchdog

    def make(default_s, rank=0):
        return real(1.5, rank, exit_fn=codes.append, poll_s=0.05, first_timeout_s=30.0)

    monkeypatch.setattr(trmod.StepWatchdog, "from_env", staticmethod(make))
    tr = Trainer(TrainConfig(model="llama-tiny", method="lora", batch_size=1, seq_len=16, synthetic=True,
                             max_steps=1, log_interval=1, checkpoint_path=str(tmp_path), device="cpu"))
    orig = tr.save_artifacts

    def slow_save():
        # 3x the step timeout.  One step: it runs under the first-step limit (30 s), so a CPU step slowed by
        # xdist load cannot trip the 1.5 s limit before the save phase begins
        time.sleep(4.5)
        return orig()

    tr.save_artifacts = slow_save
    tr.run()
    tr.close()
    assert codes == []
    assert (tmp_path / "adapter_config.json").exists()


def _bcast_worker(rank, world, port, tmp, q):
    _rank_env(rank, world, port, tmp)
    info = pdist.init_distributed("cpu")
    st = None
    if rank == 0:
        st = {"step": 7, "params": torch.arange(6, dtype=torch.float32).view(2, 3),
              "opt": {"m": torch.full((4,), 0.5, dtype=torch.bfloat16), "mask": torch.tensor([True, False]),
                      "count": 3, "tags": ["a", ("b", 2)]},
              "data": {"epoch": 1, "cursor": torch.tensor(11, dtype=torch.int64)}}
    out = pdist.broadcast_state(st, info)
    q.put((rank, out))
    pdist.destroy(info)
    _hold(tmp, port)


def test_broadcast_state_gloo(tmp_path):
    res = _run_ranks(_bcast_worker, 2, tmp_path)
    a, b = res[0], res[1]
    assert b["step"] == 7 and b["opt"]["count"] == 3 and b["opt"]["tags"] == ["a", ("b", 2)]
    for x, y in ((a["params"], b["params"]), (a["opt"]["m"], b["opt"]["m"]), (a["opt"]["mask"], b["opt"]["mask"]),
                 (a["data"]["cursor"], b["data"]["cursor"])):
        assert x.dtype == y.dtype and x.shape == y.shape and torch.equal(x, y)


def _resume_rank_worker(rank, world, port, tmp, q):
    """Phase 1 writes a resume point on rank 0's volume only; phase 2 resumes from it with rank 1
    on an empty volume; phase 3 is the same run uninterrupted."""
    torch.set_num_threads(1)
    out = {}
    base = dict(model="llama-tiny", method="lora", batch_size=2, seq_len=16, synthetic=True, device="cpu", lr=1e-2,
                warmup_steps=0, schedule="constant", bucket_mb=0.01, save_model=False, log_interval=1)
    for phase, kw in (("p1", dict(max_steps=2, save_every=1, resume=False)),
                      ("p2", dict(max_steps=4, resume=True)),
                      ("p3", dict(max_steps=4, resume=False))):
        _rank_env(rank, world, port, tmp)
        os.environ["FTC_INIT_METHOD"] = f"file://{tmp}/rdv_{port}_{phase}"
        d = os.path.join(tmp, "p3" if phase == "p3" else "job", f"rank{rank}")  # pod-local volumes
        tr = Trainer(TrainConfig(checkpoint_path=d, **base, **kw))
        tr.run()
        out[phase] = (tr.opt.export_params().clone(), tr.opt.step_count, sorted(os.listdir(d)))
        tr.close()
    q.put((rank, out))
    _hold(tmp, port)


def test_resume_from_a_checkpoint_only_rank0_holds(tmp_path):
    res = _run_ranks(_resume_rank_worker, 2, tmp_path)
    assert "checkpoint_step1.pt" in res[0]["p1"][2] and not any(f.startswith("checkpoint") for f in res[1]["p1"][2])
    # rank 1 started from rank 0's step-1 state (broadcast): both ranks agree with the uninterrupted run
    for r in (0, 1):
        p2, n2, _ = res[r]["p2"]
        p3, n3, _ = res[r]["p3"]
        assert n2 == n3 == 4
        torch.testing.assert_close(p2, p3, atol=1e-6, rtol=1e-5)
    torch.testing.assert_close(res[0]["p2"][0], res[1]["p2"][0], atol=0, rtol=0)


@pytest.mark.slow
def test_lost_peer_job_restarts_and_completes(tmp_path):
    """2 pods (Master + Worker), rank 1 hangs at step 3 outside any collective -- to rank 0 a lost
    RCCL peer.  Rank 0's collective times out (FTC_COLLECTIVE_TIMEOUT_S) and its pod fails; rank 1's
    step watchdog ends it with 124; the operator restarts both pods (backoffLimit), rank 0's step-2
    checkpoint is broadcast to rank 1's empty volume, and the job completes."""
    from fastapi.testclient import TestClient

    from finetune_controller_amd.controlplane.api.app import create_app
    from finetune_controller_amd.controlplane.context import AppContext
    from finetune_controller_amd.controlplane.spec.models.builtin import LMTrainingArguments
    from test_e2e_fakecluster import GPT2TinyFT2Node, run_monitor, wait_for

    class GPT2TinyFaulty(GPT2TinyFT2Node):
        name: str = "GPT2-tiny-FT-2node-ckpt"
        training_arguments: LMTrainingArguments = LMTrainingArguments(
            batch_size=2, seq_len=64, lr=1e-3, max_steps=6, log_interval=1, warmup_steps=1, save_every=2)

    ctx = AppContext.local(workdir=str(tmp_path), run_processes="cpu")
    ctx.registry.register(GPT2TinyFaulty)
    ctx.kube.sync_interval = 0.2
    app = create_app(ctx, run_monitor=False, force_auth=False)
    with TestClient(app) as c:
        files = {"dataset": ("corpus.txt", ("sphinx of black quartz judge my vow\n" * 300).encode(), "text/plain")}
        r = c.post("/api/v1/jobs", data={"job_name": "lost-peer", "model": "GPT2-tiny-FT-2node-ckpt", "device": "cpu",
                                        "task": "causal_lm"}, files=files)
        assert r.status_code == 200, r.text
        jid = r.json()["job_id"]
        ctx.kube.inject_fault(jid, "hang@3:rank=1", collective_timeout_s=6, step_timeout_s=12)
        ctx.kube.start(tick=0.1)
        try:
            def done():
                run_monitor(ctx)
                return c.get(f"/api/v1/jobs/{jid}").json()["status"] in ("completed", "failed")

            wait_for(done, timeout=420, step=1.5)
        finally:
            ctx.kube.stop()
        # the monitor deletes finished jobs' pods: their logs are kept in deleted_pod_logs
        logs = "\n".join("\n".join(p.logs) for p in ctx.kube.pods.values()) + \
            "\n".join("\n".join(v) for v in ctx.kube.deleted_pod_logs.values())
        assert c.get(f"/api/v1/jobs/{jid}").json()["status"] == "completed", logs[-4000:]
        assert "[fault] injected hang at step 3 on rank 1" in logs
        assert "[watchdog] rank 1: no progress" in logs
        assert "broadcasting it" in logs or "resumed from checkpoint_step2.pt" in logs
        assert [t for j, t in ctx.kube.history if j == jid].count("Restarting") >= 2  # both pods
        m = c.get(f"/api/v1/jobs/{jid}/metrics").json()["metrics"]
        assert max(int(row["step"]) for row in m) == 6
        # the sidecar ships the artifacts, never the resume checkpoints that live on the pod's volume
        keys = [o.Key for o in ctx.objects.list(ctx.s3.bucket, "finetune_jobs/")]
        assert any(k.endswith("metrics.csv") for k in keys)
        assert not any("checkpoint_step" in k or k.endswith(".tmp") for k in keys), keys


def test_first_write_registry_flushes_unwritten_weight():
    """ops.linear first-write gradients: a registered projection weight that a step leaves unwritten is
    zeroed by flush_fresh through its CURRENT main_grad (the registry holds only a weak reference), a
    dead parameter is skipped, and a new optimizer resets the registry."""
    from finetune_controller_amd.ops import linear as L

    prior = L._FIRST_WRITE
    try:
        L.set_first_write(True)
        p = torch.nn.Parameter(torch.zeros(4, 4))
        p.main_grad = torch.zeros(4, 4)
        assert L.take_fresh(p, p.main_grad) == 1.0  # first sight: registered, zeroed this step
        assert L.is_grad_owned(p)
        L.mark_fresh([id(p)])  # the optimizer skipped zeroing it
        p.main_grad = torch.full((4, 4), 3.0)  # a re-homed buffer: the flush must use the current one
        L.gradients_final()  # nothing wrote it this step
        assert torch.count_nonzero(p.main_grad) == 0
        L.mark_fresh([id(p)])
        assert L.take_fresh(p, p.main_grad) == 0.0  # written by a beta = 0 GEMM: no flush needed
        q = torch.nn.Parameter(torch.zeros(2))
        q.main_grad = torch.zeros(2)
        L.take_fresh(q, q.main_grad)
        L.mark_fresh([id(q)])
        del q
        L.flush_fresh()  # dead parameter: skipped
        from finetune_controller_amd.train.optim import FlatAdamW

        FlatAdamW([torch.nn.Parameter(torch.zeros(8))])
        assert not L.is_grad_owned(p)
    finally:
        L.set_first_write(prior)
