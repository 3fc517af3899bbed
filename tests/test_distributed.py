"""Multi-process paths on CPU (gloo): the bench launcher, fp32 gradient accumulation under data
parallelism, and resume across world sizes / ZeRO settings.

These are the CPU rehearsals of what the driver's 8-GPU run exercises with RCCL: the process layout,
rendezvous, bucketed reductions and the rank-0 JSON contract are identical; only the transport
differs."""
import json
import math
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.multiprocessing as mp

from finetune_controller_amd.models import checkpoint as ckpt
from finetune_controller_amd.parallel import dist as pdist
from finetune_controller_amd.train.data import SyntheticTokens
from finetune_controller_amd.train.trainer import TrainConfig, Trainer

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank_env(rank, world, port, tmp):
    # file rendezvous in the test dir: a picked-then-released TCP port can be taken by a parallel test
    os.environ["FTC_INIT_METHOD"] = f"file://{tmp}/rdv_{port}"
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)


def _hold(tmp, port, timeout=180.0):
    """Keep a rank alive until the parent has read its queued tensors (they travel by fd)."""
    import time

    t0 = time.time()
    while not os.path.exists(os.path.join(tmp, f"release_{port}")) and time.time() - t0 < timeout:
        time.sleep(0.05)


def _run_ranks(target, world, tmp, *args, timeout=240):
    port = _port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=target, args=(r, world, port, str(tmp), q, *args)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = dict(q.get(timeout=timeout) for _ in range(world))
    finally:
        open(os.path.join(str(tmp), f"release_{port}"), "w").close()
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    return res


# --------------------------------------------------------------------------- bench.py launcher
@pytest.mark.slow
def test_bench_self_launches_ranks_on_cpu(tmp_path):
    """``python bench.py --gpus 2`` without torchrun spawns 2 ranks (gloo on CPU here), prints exactly
    one JSON line from rank 0 with n_gpus == world size seen by the process group == 2."""
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "FTC_INIT_METHOD"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
                        "--device", "cpu", "--model", "llama-tiny", "--batch-size", "2", "--seq-len", "32",
                        "--launcher-timeout", "240"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["world_size_pg"] == 2 and out["dist_backend"] == "gloo"
    assert out["config"]["parallelism"] == "dp2" and out["config"]["global_batch"] == 4
    assert out["value"] > 0 and out["steps"] == 2 and out["warmup"] == 1
    assert out["rank_ms_per_step"]["max"] >= out["rank_ms_per_step"]["min"] > 0
    assert out["comm"]["collective_timeout_s"] == 300
    # the transport diagnostics come after the headline, as one JSON object on stderr
    diag = [json.loads(ln)["diagnostics"] for ln in r.stderr.splitlines() if ln.startswith('{"diagnostics"')]
    assert len(diag) == 1 and diag[0]["torch"]["busbw_GBps"] > 0 and not diag[0].get("abandoned")
    assert out["comm"]["n_buckets"] >= 1 and out["comm"]["wire_GB_per_step"] > 0
    assert out["comm"]["comm_exposed_ms"] is None  # device events: GPU runs only


@pytest.mark.slow
def test_bench_eight_ranks_on_cpu(tmp_path):
    """The driver's 8-GPU command shape, rehearsed with 8 gloo ranks: exactly one JSON line, n_gpus ==
    the process group's world size == 8, global batch 8 x micro-batch."""
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "FTC_INIT_METHOD"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--steps", "1", "--warmup", "1",
                        "--device", "cpu", "--model", "llama-tiny", "--batch-size", "1", "--seq-len", "16",
                        "--launcher-timeout", "400"],
                       capture_output=True, text=True, timeout=480, env=env, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 8 and out["world_size_pg"] == 8
    assert out["config"]["parallelism"] == "dp8" and out["config"]["global_batch"] == 8
    assert out["config"]["zero_stage"] == 0  # LoRA: plain bucketed all-reduce


@pytest.mark.slow
def test_bench_headline_survives_a_stalled_diagnostic(tmp_path):
    """VERDICT r5 Next #3: rank 3 parks inside the post-headline sweep (fault hook).  The headline line is
    still on stdout, every rank abandons the sweep at the diagnostic budget and exits 0, and the whole run
    ends within the budget instead of a collective timeout."""
    import time as _time

    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1", FTC_BENCH_DIAG_STALL_RANK="3")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "FTC_INIT_METHOD",
              "FTC_COLLECTIVE_TIMEOUT_S"):
        env.pop(k, None)
    t0 = _time.monotonic()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--steps", "1", "--warmup", "1",
                        "--device", "cpu", "--model", "llama-tiny", "--batch-size", "1", "--seq-len", "16",
                        "--launcher-timeout", "400", "--diag-budget", "15"],
                       capture_output=True, text=True, timeout=480, env=env, cwd=str(tmp_path))
    wall = _time.monotonic() - t0
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 8 and out["value"] > 0
    diag = [json.loads(ln)["diagnostics"] for ln in r.stderr.splitlines() if ln.startswith('{"diagnostics"')]
    assert len(diag) == 1 and diag[0]["abandoned"] is True and "torch" not in diag[0]
    assert 15 <= diag[0]["elapsed_s"] < 40
    # the stall costs the budget, not the 60 s group timeout or the 300 s default-group timeout
    assert wall < 300, wall


@pytest.mark.slow
def test_bench_eight_ranks_full_ft_zero1_on_cpu(tmp_path):
    """The 8-rank command for full fine-tuning: ZeRO-1 by default, with the parameter all-gather overlapped
    with the next forward and its exposed time reported beside the gradient reduction's (device events:
    None on CPU, a number on the GPU)."""
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "FTC_INIT_METHOD"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--steps", "2", "--warmup", "1",
                        "--device", "cpu", "--model", "llama-tiny", "--method", "full", "--batch-size", "1",
                        "--seq-len", "16", "--launcher-timeout", "400"],
                       capture_output=True, text=True, timeout=480, env=env, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.strip()][-1])
    assert out["n_gpus"] == 8 and out["config"]["zero_stage"] == 1
    assert out["config"]["parallelism"] == "dp8-zero1"
    assert "param_sync_exposed_ms" in out["comm"] and out["comm"]["param_sync_exposed_ms"] is None
    assert out["comm"]["zero_gather_overlap"] is True
    # the fields that make the first 8-GPU record explain itself (RCCL's channel count: None over gloo)
    assert "rccl_channels" in out and out["rccl_channels"] is None
    assert out["comm"]["grad_wire"] == "float32"


@pytest.mark.slow
def test_bench_eight_ranks_full_ft_bf16_wire_on_cpu(tmp_path):
    """``--grad-wire bf16`` (VERDICT r4 Next #5) on the 8-rank full-FT command: fp32 gradient buffer, bf16
    reduce-scatter -- (2 + p) / (4 + p) of the fp32 wire's bytes per step (p = the all-gathered parameter's
    bytes: 4 / 6 for the bf16 model on the GPU), same loss as the fp32 wire to bf16 precision, and --rccl-channels reaches the RCCL env."""
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "FTC_INIT_METHOD"):
        env.pop(k, None)
    outs = {}
    for wire in ("auto", "bf16"):
        r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--steps", "2", "--warmup",
                            "1", "--device", "cpu", "--model", "llama-tiny", "--method", "full", "--batch-size", "1",
                            "--seq-len", "16", "--launcher-timeout", "400", "--grad-wire", wire, "--rccl-channels", "4"],
                           capture_output=True, text=True, timeout=480, env=env, cwd=str(tmp_path))
        assert r.returncode == 0, r.stderr[-3000:]
        outs[wire] = json.loads([ln for ln in r.stdout.splitlines() if ln.strip()][-1])
    a, b = outs["auto"], outs["bf16"]
    assert a["config"]["grad_dtype"] == b["config"]["grad_dtype"] == "float32"
    assert a["comm"]["grad_wire"] == "float32" and b["comm"]["grad_wire"] == "bfloat16"
    pb = 4 if b["dtype"] == "fp32" else 2  # parameter bytes of the all-gather (the CPU rehearsal trains in fp32)
    assert abs(b["comm"]["wire_GB_per_step"] / a["comm"]["wire_GB_per_step"] - (2 + pb) / (4 + pb)) < 0.02
    assert abs(a["loss"] - b["loss"]) < 2e-2 * abs(a["loss"])
    assert b["comm"]["env"]["NCCL_MIN_NCHANNELS"] == b["comm"]["env"]["NCCL_MAX_NCHANNELS"] == "4"


def _zero_overlap_worker(rank, world, port, tmp, q, overlap):
    os.environ["FTC_ZERO_GATHER_OVERLAP"] = "1" if overlap else "0"
    _rank_env(rank, world, port, tmp)
    tc = TrainConfig(model="llama-tiny", method="full", batch_size=2, seq_len=16, synthetic=True, max_steps=3,
                     checkpoint_path=tmp, resume=False, device="cpu", dtype="bf16", lr=1e-2, bucket_mb=0.05,
                     max_grad_norm=1.0, save_model=False, zero_stage=1, weight_decay=0.1)
    tr = Trainer(tc)
    gated = tr.model.param_gate is not None
    losses = [float(tr.train_step(1e-2)) for _ in range(3)]
    pending = len(tr.opt._pending)  # the last step's gathers, waited for by the next forward / join
    q.put((rank, {"losses": losses, "params": tr.opt.export_params().float().clone(), "gated": gated,
                  "buckets": len(tr.opt.buckets), "pending": pending}))
    tr.close()
    _hold(tmp, port)


@pytest.mark.slow
def test_zero1_overlapped_gather_matches_synchronous(tmp_path):
    """ZeRO-1 with each bucket's parameter all-gather issued after its own update and the next forward
    gated per layer (ShardedFlatAdamW.enable_gather_overlap) trains exactly like the synchronous gather:
    equal losses and parameters after three steps on 2 gloo ranks with several buckets."""
    ov = _run_ranks(_zero_overlap_worker, 2, tmp_path, True)
    sy = _run_ranks(_zero_overlap_worker, 2, tmp_path, False)
    assert ov[0]["gated"] and not sy[0]["gated"]
    assert ov[0]["buckets"] > 2 and ov[0]["pending"] > 0 and sy[0]["pending"] == 0
    for r in (0, 1):
        assert ov[r]["losses"] == sy[r]["losses"]
        torch.testing.assert_close(ov[r]["params"], sy[r]["params"], atol=0, rtol=0)
    torch.testing.assert_close(ov[0]["params"], ov[1]["params"], atol=0, rtol=0)


def test_device_key_prefers_pci_location(monkeypatch):
    """Two cards that report one UUID (seen in some containerised setups) still get distinct keys from
    their PCI location; without PCI fields the UUID, then the index, is used."""
    from types import SimpleNamespace

    props = {0: SimpleNamespace(uuid="same", pci_domain_id=0, pci_bus_id=0x11, pci_device_id=0),
             1: SimpleNamespace(uuid="same", pci_domain_id=0, pci_bus_id=0x21, pci_device_id=0),
             2: SimpleNamespace(uuid="u2"), 3: SimpleNamespace(uuid="")}
    monkeypatch.setattr(torch.cuda, "get_device_properties", lambda d: props[d.index])
    keys = [pdist.device_key(torch.device("cuda", i)) for i in range(4)]
    assert keys[0] != keys[1] and keys[0].startswith("pci:0:11:0/")
    assert keys[2] == "u2" and keys[3] == "index3"


@pytest.mark.gpu
def test_device_key_on_the_gpu():
    key = pdist.device_key(torch.device("cuda", 0))
    print("device key:", key)
    assert key.startswith("pci:"), key  # this image's torch reports the PCI location


def test_distinct_device_binding_checks(monkeypatch):
    from finetune_controller_amd.parallel import dist as pdist

    for k in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "LOCAL_WORLD_SIZE"):
        monkeypatch.delenv(k, raising=False)

    pdist.check_distinct_devices([("h0", "g0", 0), ("h0", "g1", 1), ("h1", "g0", 2)])  # per host: distinct
    with pytest.raises(RuntimeError, match="ranks 0 and 2"):
        pdist.check_distinct_devices([("h0", "g0", 0), ("h0", "g1", 1), ("h0", "g0", 2)])
    pdist.check_local_rank(7, 8)
    with pytest.raises(RuntimeError, match="LOCAL_RANK 8"):
        pdist.check_local_rank(8, 8)
    assert pdist.local_device_index(5, 8) == 5
    # one visible device: rank 5 binds it only when the launcher narrowed the visible set to it ...
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    with pytest.raises(RuntimeError, match="LOCAL_RANK 5"):  # torchrun x8 on a 1-GPU host: fail early
        pdist.local_device_index(5, 1)
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "5")
    assert pdist.local_device_index(5, 1) == 0
    monkeypatch.delenv("HIP_VISIBLE_DEVICES")
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "1")  # ... or the node runs one rank
    assert pdist.local_device_index(0, 1) == 0
    assert pdist.local_device_index(5, 2, share=True) == 1
    with pytest.raises(RuntimeError, match="LOCAL_RANK 4"):
        pdist.local_device_index(4, 4)


def test_bench_refuses_mislabelled_world(tmp_path):
    env = dict(os.environ, PYTHONPATH=ROOT, WORLD_SIZE="3", RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--device", "cpu"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=str(tmp_path))
    assert r.returncode == 2 and "WORLD_SIZE=3" in r.stderr


def test_bench_launcher_propagates_rank_failure(tmp_path):
    """A failing rank ends the launcher with a non-zero code (here: an unknown model on every rank)."""
    env = dict(os.environ, PYTHONPATH=ROOT)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--device", "cpu",
                        "--model", "no-such-model", "--launcher-timeout", "120"],
                       capture_output=True, text=True, timeout=180, env=env, cwd=str(tmp_path))
    assert r.returncode != 0 and not r.stdout.strip()


# --------------------------------------------------------------------------- fp32 grad accumulation
ACCUM = 4


def _accum_worker(rank, world, port, tmp, q, grad_dtype, zero, grad_wire="auto"):
    _rank_env(rank, world, port, tmp)
    tc = TrainConfig(model="llama-tiny", method="full", batch_size=2, seq_len=16, synthetic=True, max_steps=1,
                     checkpoint_path=tmp, resume=False, device="cpu", dtype="bf16", lr=0.0, bucket_mb=0.05,
                     max_grad_norm=0.0, save_model=False, grad_accum=ACCUM, grad_dtype=grad_dtype, zero_stage=zero,
                     grad_wire=grad_wire)
    tr = Trainer(tc)
    tr.train_step(0.0)
    out = {"dtype": str(tr.opt.grad_flat.dtype), "buckets": len(tr.ddp.buckets), "zero": tr.zero_stage,
           "offsets": [tuple(o) for o in tr.opt.offsets], "numel": tr.opt.numel,
           "wire": tr.ddp.wire_bytes_per_step()}
    if tr.zero_stage:  # this rank's owned slices of the summed gradient
        out["shard"] = tr.opt.grad_shard.detach().double().clone()
        out["ranges"] = list(tr.opt.shard_ranges)
        out["shard_offsets"] = list(tr.opt.shard_offsets)
    else:
        out["grad"] = tr.opt.grad_flat.detach().double().clone()
    q.put((rank, out))
    tr.close()
    _hold(tmp, port)


def _reference_grads(tmp, world):
    """Single process: every (rank, micro-batch) gradient computed alone (bf16 model, same weights and
    data as the ranks), summed in float64; returned per parameter in layout order."""
    total = None
    for rank in range(world):
        tc = TrainConfig(model="llama-tiny", method="full", batch_size=2, seq_len=16, synthetic=True, max_steps=1,
                         checkpoint_path=str(tmp), resume=False, device="cpu", dtype="bf16", lr=0.0,
                         max_grad_norm=0.0, save_model=False, grad_accum=1, grad_dtype="fp32", seed=1)
        tr = Trainer(tc)
        tr._data = SyntheticTokens(tr.cfg.vocab_size, 2, 16, "cpu", seed=1 + rank)
        tr.steps_per_epoch = 100
        for _ in range(ACCUM):
            tr.train_step(0.0)  # lr 0, no decay: the weights stay put
            g = tr.opt.grad_flat.detach().double().clone()
            total = g if total is None else total + g
        layout = [(o, n) for o, n in tr.opt.offsets]
        tr.close()
    return torch.cat([total[o:o + n] for o, n in layout])


def _summed_grads(res, world):
    """The reduced gradient per parameter (layout order) as the ranks hold it: the all-reduced flat
    buffer (identical on every rank), or the ZeRO-1 owned slices put back together."""
    r0 = res[0]
    if not r0["zero"]:
        for r in range(1, world):
            torch.testing.assert_close(res[r]["grad"], r0["grad"], atol=0, rtol=0)  # all ranks hold the same sum
        flat = r0["grad"]
    else:
        flat = torch.zeros(r0["numel"], dtype=torch.float64)
        for r in range(world):
            sh = res[r]["shard"]
            for (lo, hi), o in zip(res[r]["ranges"], res[r]["shard_offsets"]):
                flat[lo:hi] = sh[o:o + hi - lo]
    return torch.cat([flat[o:o + n] for o, n in r0["offsets"]])


@pytest.mark.slow
def test_fp32_grad_accumulation_three_ranks_matches_fp64_reference(tmp_path):
    """3 gloo ranks x grad_accum 4 on a bf16 full fine-tune: the fp32 gradient (accumulated across
    micro-batches, reduced across ranks) equals the float64 sum of the 12 per-micro-batch gradients to
    fp32 rounding -- on the default path (auto = ZeRO-1: fp32 reduce-scatter into owned slices) and on
    the plain fp32 all-reduce; the bf16 buffer is measurably worse.  ZeRO-1 moves 3/4 of the all-reduce's
    bytes (fp32 reduce-scatter + bf16 all-gather vs fp32 all-reduce)."""
    world = 3
    ref = _reference_grads(tmp_path, world)
    errs, wire = {}, {}
    for gd, zero in (("auto", -1), ("fp32", 0), ("bf16", 0)):
        res = _run_ranks(_accum_worker, world, tmp_path, gd, zero)
        assert res[0]["zero"] == (1 if zero == -1 else 0)
        g = _summed_grads(res, world)
        assert res[0]["dtype"] == ("torch.bfloat16" if gd == "bf16" else "torch.float32")
        assert res[0]["buckets"] > 1
        errs[(gd, zero)] = float((g - ref).abs().max() / ref.abs().max())
        wire[(gd, zero)] = res[0]["wire"]
    assert errs[("auto", -1)] < 2e-6 and errs[("fp32", 0)] < 2e-6, errs
    assert errs[("bf16", 0)] > 20 * errs[("fp32", 0)], errs
    assert abs(wire[("auto", -1)] / wire[("fp32", 0)] - 0.75) < 0.02, wire


@pytest.mark.slow
def test_bf16_grad_wire_three_ranks_bounded_against_fp64(tmp_path):
    """``grad_wire=bf16`` under ZeRO-1 (VERDICT r4 Next #5): the fp32 buffer accumulates the 4 micro-batches
    exactly on each rank, only the reduce-scatter travels as bf16.  3 gloo ranks x accumulation 4 against
    the float64 sum: the error is bounded by a few bf16 ulps of the largest gradient (one rounding per
    rank's partial + the ring's bf16 adds), no worse than a bf16 buffer (which also rounds every
    accumulation), and the gradient reduction moves half the bytes of the fp32 reduce-scatter."""
    world = 3
    ref = _reference_grads(tmp_path, world)
    res = _run_ranks(_accum_worker, world, tmp_path, "auto", -1, "bf16")
    assert res[0]["zero"] == 1 and res[0]["dtype"] == "torch.float32" and res[0]["buckets"] > 1
    err_wire = float((_summed_grads(res, world) - ref).abs().max() / ref.abs().max())
    wire_bf16 = res[0]["wire"]
    res = _run_ranks(_accum_worker, world, tmp_path, "auto", -1, "auto")
    err_fp32 = float((_summed_grads(res, world) - ref).abs().max() / ref.abs().max())
    wire_fp32 = res[0]["wire"]
    res = _run_ranks(_accum_worker, world, tmp_path, "bf16", -1, "auto")
    err_buf = float((_summed_grads(res, world) - ref).abs().max() / ref.abs().max())
    assert err_fp32 < 2e-6, err_fp32
    assert 2e-6 < err_wire < 1.2e-2, err_wire  # bf16 epsilon 7.8e-3: at most ~1.5 ulp of the largest entry
    assert err_wire <= 1.5 * err_buf, (err_wire, err_buf)
    # fp32 reduce-scatter (4 B) + bf16 gather (2 B) -> bf16 + bf16: 4 / 6 of the bytes
    assert abs(wire_bf16 / wire_fp32 - 4 / 6) < 0.02, (wire_bf16, wire_fp32)


def test_grad_wire_rejects_unsupported_pairs():
    tc = TrainConfig(model="llama-tiny", method="lora", batch_size=1, seq_len=16, synthetic=True, device="cpu",
                     dtype="bf16", save_model=False, resume=False, grad_wire="fp8")
    with pytest.raises(ValueError, match="grad_wire"):
        Trainer(tc)


def test_grad_dtype_auto_policy():
    tc = TrainConfig(model="llama-tiny", method="full", batch_size=1, seq_len=16, synthetic=True, device="cpu",
                     dtype="bf16", grad_accum=2, save_model=False, resume=False)
    tr = Trainer(tc)
    assert tr.opt.grad_flat.dtype == torch.float32
    tr.train_step(1e-3)  # the fold hooks leave no model-dtype .grad behind
    assert all(p.grad is None for p in tr.opt.params)
    tr.close()
    tc.grad_accum, tc.method = 1, "lora"
    tr = Trainer(tc)
    assert tr.opt.grad_flat.dtype == torch.bfloat16
    tr.close()


# --------------------------------------------------------------------------- resume across layouts
def _resume_worker(rank, world, port, tmp, q, zero):
    _rank_env(rank, world, port, tmp)
    tc = TrainConfig(model="llama-tiny", method="lora", batch_size=2, seq_len=16, synthetic=True, max_steps=2,
                     checkpoint_path=tmp, resume=False, device="cpu", lr=1e-2, warmup_steps=0, bucket_mb=0.01,
                     save_model=False, zero_stage=zero, weight_decay=0.1)
    tr = Trainer(tc)
    for _ in range(2):
        tr.train_step(1e-2)
    tr.step = 2
    tr.save_resume()  # collective under ZeRO-1; rank 0 writes checkpoint_step2.pt
    q.put((rank, {"params": tr.opt.export_params().clone(), "padded": tr.opt.numel}))
    tr.close()
    _hold(tmp, port)


@pytest.mark.slow
def test_resume_zero1_world3_checkpoint_at_world1(tmp_path):
    """A checkpoint written by 3 ZeRO-1 ranks (buckets padded to a multiple of 3) resumes in a
    1-process run without ZeRO: same trainable parameters, moments and step."""
    res = _run_ranks(_resume_worker, 3, tmp_path, 1)
    path = os.path.join(str(tmp_path), "checkpoint_step2.pt")
    st = torch.load(path, map_location="cpu", weights_only=True)
    tc = TrainConfig(model="llama-tiny", method="lora", batch_size=2, seq_len=16, synthetic=True, max_steps=4,
                     checkpoint_path=str(tmp_path), device="cpu", lr=1e-2, save_model=False)
    tr = Trainer(tc)
    assert tr.opt.numel != res[0]["padded"]  # the two layouts really differ
    ckpt.load_resume(path, tr.opt)
    torch.testing.assert_close(tr.opt.export_params(), res[0]["params"], atol=0, rtol=0)
    sd = tr.opt.state_dict()
    for k in ("master", "exp_avg", "exp_avg_sq"):
        torch.testing.assert_close(sd[k], st["opt"][k], atol=0, rtol=0)
    assert tr.opt.step_count == 2
    tr.train_step(1e-2)  # and it keeps training
    tr.close()


def test_resume_rejects_foreign_parameter_set(tmp_path):
    base = dict(model="llama-tiny", batch_size=1, seq_len=16, synthetic=True, device="cpu", save_model=False,
                checkpoint_path=str(tmp_path), resume=False)
    tr = Trainer(TrainConfig(method="lora", lora_r=8, **base))
    tr.step = 1
    tr.save_resume()
    tr.close()
    tr = Trainer(TrainConfig(method="lora", lora_r=4, **base))
    with pytest.raises(ValueError):
        ckpt.load_resume(os.path.join(str(tmp_path), "checkpoint_step1.pt"), tr.opt)
    tr.close()


# --------------------------------------------------------------------------- Ulysses sequence parallelism
def _sp_worker(rank, world, port, tmp, q, method, window_model, doc_len, batch=2):
    _rank_env(rank, world, port, tmp)
    tc = TrainConfig(model=window_model, method=method, batch_size=batch, seq_len=64, synthetic=True, max_steps=1,
                     checkpoint_path=tmp, resume=False, device="cpu", dtype="fp32", lr=0.0, max_grad_norm=0.0,
                     save_model=False, sp=world, bucket_mb=0.05, synthetic_doc_len=doc_len, eval_batches=2)
    tr = Trainer(tc)
    loss = tr.train_step(0.0)
    q.put((rank, {"loss": float(loss), "grad": tr.opt.grad_flat.detach().double().clone(),
                  "layout": [(o, n) for o, n in tr.opt.offsets], "eval": tr.evaluate()}))
    tr.close()
    _hold(tmp, port)


@pytest.mark.slow
@pytest.mark.parametrize("method,model,doc_len,batch", [("full", "llama-tiny", 0, 2), ("lora", "llama-tiny", 0, 2),
                                                        ("full", "mistral-tiny", 0, 2), ("full", "llama-tiny", 40, 2),
                                                        ("lora", "llama-tiny", 0, 1)])
def test_sequence_parallel_matches_single_process(tmp_path, method, model, doc_len, batch):
    """Ulysses SP over 2 gloo ranks (each holds half of every sequence; attention all-to-alls heads <->
    tokens) against one process training the same full sequences: the mean of the ranks' losses and the
    all-reduced gradient equal the single-process loss / gradient (fp32, sliding window included), also
    when masked labels leave the two halves different valid-token counts (doc_len 40: the document
    boundary's masked label falls in the second half only), and the held-out loss matches.  batch 1
    takes the all-to-all path without the token-major reorder copies."""
    world = 2
    res = _run_ranks(_sp_worker, world, tmp_path, method, model, doc_len, batch)
    tc = TrainConfig(model=model, method=method, batch_size=batch, seq_len=64, synthetic=True, max_steps=1,
                     checkpoint_path=str(tmp_path), resume=False, device="cpu", dtype="fp32", lr=0.0,
                     max_grad_norm=0.0, save_model=False, synthetic_doc_len=doc_len, eval_batches=2)
    tr = Trainer(tc)
    ref_loss = float(tr.train_step(0.0))
    ref = tr.opt.grad_flat.detach().double().clone()
    ref_eval = tr.evaluate()
    tr.close()
    assert abs(sum(res[r]["loss"] for r in range(world)) / world - ref_loss) < 1e-5 * abs(ref_loss)
    assert res[0]["eval"] == res[1]["eval"]
    assert abs(res[0]["eval"] - ref_eval) < 1e-5 * abs(ref_eval), (res[0]["eval"], ref_eval)
    g = res[0]["grad"]
    torch.testing.assert_close(res[1]["grad"], g, atol=0, rtol=0)  # one all-reduced gradient
    # the buffer holds the SUM of the ranks' half-sequence mean gradients; the optimizer applies
    # grad_scale = 1/world, which makes it the gradient of the whole batch's mean loss
    torch.testing.assert_close(g / world, ref, atol=1e-6 * ref.abs().max().item(), rtol=1e-4)


# --------------------------------------------------------------------------- SP over RCCL on the GPU
_SP_GPU = dict(model="llama3-8b-1l", batch_size=2, seq_len=1024, synthetic=True, max_steps=1, resume=False,
               device="cuda", dtype="bf16", lr=0.0, max_grad_norm=0.0, save_model=False, grad_dtype="fp32")


def _grad_digest(tr):
    """A fixed random sample of the flat fp32 gradient (the whole buffer is GBs for full FT) + its norm."""
    g = tr.opt.grad_flat.detach()
    gen = torch.Generator().manual_seed(1234)
    idx = torch.randint(0, g.numel(), (1 << 20,), generator=gen)
    return g[idx.to(g.device)].float().cpu(), float(g.double().norm())


def _sp_gpu_worker(rank, world, port, tmp, q, method):
    os.environ["FTC_SHARE_GPU"] = "1"  # both ranks on the box's one card, RCCL over loopback
    _rank_env(rank, world, port, tmp)
    tr = Trainer(TrainConfig(method=method, checkpoint_path=tmp, sp=world, **_SP_GPU))
    loss = float(tr.train_step(0.0))
    sample, norm = _grad_digest(tr)
    q.put((rank, {"loss": loss, "sample": sample, "norm": norm}))
    tr.close()
    _hold(tmp, port)


@pytest.mark.gpu
@pytest.mark.parametrize("method", ["lora", "full"])
def test_sequence_parallel_rccl_matches_single_gpu(tmp_path, method):
    """Ulysses SP with 2 ranks over RCCL (sharing the box's card) on a Llama-3-8B-geometry layer, bf16 on
    the HIP kernels (flash attention over the full 1024-token sequence for 16 of the 32 heads per rank),
    against one process on the whole sequences: same mean loss, one all-reduced gradient on both ranks,
    and a gradient equal to the single-process one up to bf16 re-association (the token halves reduce
    in two GEMMs + an all-reduce instead of one GEMM)."""
    res = _run_ranks(_sp_gpu_worker, 2, tmp_path, method, timeout=100)
    tr = Trainer(TrainConfig(method=method, checkpoint_path=str(tmp_path), **_SP_GPU))
    ref_loss = float(tr.train_step(0.0))
    ref, ref_norm = _grad_digest(tr)
    tr.close()
    loss = (res[0]["loss"] + res[1]["loss"]) / 2
    assert abs(loss - ref_loss) < 1e-4 * abs(ref_loss), (loss, ref_loss)
    torch.testing.assert_close(res[1]["sample"], res[0]["sample"], atol=0, rtol=0)
    g = res[0]["sample"] / 2  # the buffer holds the sum over ranks; the optimizer scales by 1/world
    assert ref.abs().max() > 0
    cos = torch.nn.functional.cosine_similarity(g.double(), ref.double(), dim=0).item()
    print(f"sp2 {method}: loss {loss:.6f} vs {ref_loss:.6f}, grad cos {cos:.6f}, norm {res[0]['norm'] / 2:.6g} vs "
          f"{ref_norm:.6g}")
    assert cos > 0.9999, cos  # measured 0.999995-0.999997
    assert abs(res[0]["norm"] / 2 - ref_norm) < 1e-3 * ref_norm, (res[0]["norm"] / 2, ref_norm)


# --------------------------------------------------------------------------- DDP over RCCL on the GPU
_DDP_GPU = dict(model="llama3-8b-1l", batch_size=2, seq_len=512, synthetic=True, max_steps=1, resume=False,
                device="cuda", dtype="bf16", lr=0.0, max_grad_norm=0.0, save_model=False, grad_dtype="fp32",
                zero_stage=0)  # replicated all-reduce (full FT would default to ZeRO-1: test_zero1_rccl_* below)


def _ddp_gpu_worker(rank, world, port, tmp, q, method, engine):
    os.environ["FTC_SHARE_GPU"] = "1"
    _rank_env(rank, world, port, tmp)
    from finetune_controller_amd.ops import linear as L

    # "-side": weight gradients on the side stream (the default), buckets launched behind them; plain
    # engine names pin the main-stream path
    L.set_wgrad_stream(engine.endswith("-side"))
    engine = engine.removesuffix("-side")
    tr = Trainer(TrainConfig(method=method, checkpoint_path=tmp, comm_engine=engine,
                             bucket_mb=0.25 if method == "lora" else 64.0, **_DDP_GPU))
    tr.train_step(0.0)
    sample, norm = _grad_digest(tr)
    q.put((rank, {"sample": sample, "norm": norm, "buckets": len(tr.ddp.buckets)}))
    tr.close()
    _hold(tmp, port)


@pytest.mark.gpu
@pytest.mark.parametrize("method,engine", [("lora", "torch"), ("lora", "native"), ("full", "torch"),
                                           ("full", "torch-side")])
def test_ddp_rccl_matches_per_rank_sum(tmp_path, method, engine):
    """DDP with 2 ranks over RCCL (sharing the card; torch.distributed or the native engine): the bucketed
    all-reduce -- launched from grad hooks mid-backward, including the grad-ready hook of weights whose
    gradient a beta=1 GEMM writes in place -- leaves on both ranks the sum of the gradients one process
    computes on each rank's batch alone (same kernels, same data seeds; fp32 buffer)."""
    res = _run_ranks(_ddp_gpu_worker, 2, tmp_path, method, engine, timeout=100)
    total, norm_ref = None, None
    for rank in range(2):
        tr = Trainer(TrainConfig(method=method, checkpoint_path=str(tmp_path), **_DDP_GPU))
        tr._data = SyntheticTokens(tr.cfg.vocab_size, 2, 512, tr.device, seed=tr.tc.seed + rank)
        tr.train_step(0.0)
        if total is None:
            total = tr.opt.grad_flat.detach().clone()
        else:
            total += tr.opt.grad_flat.detach()
        tr.close()
    gen = torch.Generator().manual_seed(1234)
    idx = torch.randint(0, total.numel(), (1 << 20,), generator=gen)
    ref, norm_ref = total[idx.to(total.device)].float().cpu(), float(total.double().norm())
    assert res[0]["buckets"] > 1
    torch.testing.assert_close(res[1]["sample"], res[0]["sample"], atol=0, rtol=0)
    scale = ref.abs().max().item()
    assert scale > 0
    err = (res[0]["sample"] - ref).abs().max().item() / scale
    print(f"ddp2 {method}/{engine}: max rel err {err:.3g}, norm {res[0]['norm']:.6g} vs {norm_ref:.6g}, "
          f"{res[0]['buckets']} buckets")
    assert err < 1e-5, err  # measured: bitwise equal (0) for all three


def _zero_gpu_worker(rank, world, port, tmp, q, zero):
    os.environ["FTC_SHARE_GPU"] = "1"
    _rank_env(rank, world, port, tmp)
    tr = Trainer(TrainConfig(method="full", checkpoint_path=tmp,
                             **{**_DDP_GPU, "lr": 1e-3, "max_grad_norm": 1.0, "zero_stage": zero}))
    params = [p for p in tr.model.parameters() if p.requires_grad]

    def digest():
        return torch.cat([p.detach().reshape(-1)[:: max(1, p.numel() // 4096)].float().cpu() for p in params])

    before = digest()
    tr.train_step(1e-3)
    tr._join_update()  # the overlapped parameter all-gather (waited for by the next forward otherwise)
    torch.cuda.synchronize()
    q.put((rank, {"before": before, "after": digest()}))
    tr.close()
    _hold(tmp, port)


@pytest.mark.gpu
def test_zero1_rccl_update_matches_ddp(tmp_path):
    """ZeRO-1 on 2 RCCL ranks (gradient reduce-scatter, AdamW on each rank's shard, parameter all-gather;
    grad clipping on the sharded norm) updates every parameter exactly as replicated DDP + AdamW does."""
    z = _run_ranks(_zero_gpu_worker, 2, tmp_path, 1, timeout=100)
    d = _run_ranks(_zero_gpu_worker, 2, tmp_path, 0, timeout=100)
    for r in (0, 1):
        torch.testing.assert_close(z[r]["before"], d[r]["before"], atol=0, rtol=0)
        torch.testing.assert_close(z[r]["after"], z[0]["after"], atol=0, rtol=0)  # the all-gather
    moved = (d[0]["after"] != d[0]["before"]).float().mean().item()
    diff = (z[0]["after"] - d[0]["after"]).abs().max().item()
    print(f"zero1 vs ddp: {moved:.3f} of sampled weights moved, max |diff| {diff:.3g}")
    assert moved > 0.5
    torch.testing.assert_close(z[0]["after"], d[0]["after"], atol=1e-6, rtol=0)


def _zero_wire_worker(rank, world, port, tmp, q, engine):
    os.environ["FTC_SHARE_GPU"] = "1"
    _rank_env(rank, world, port, tmp)
    from finetune_controller_amd.ops import linear as L

    L.set_wgrad_stream(True)  # dW on the side stream: the bf16 staging is allocated there
    tr = Trainer(TrainConfig(method="full", checkpoint_path=tmp, comm_engine=engine, grad_wire="bf16",
                             **{**_DDP_GPU, "max_steps": 3, "lr": 1e-3, "max_grad_norm": 1.0, "zero_stage": 1}))
    losses = [float(tr.train_step(1e-3)) for _ in range(3)]
    tr._join_update()
    torch.cuda.synchronize()
    q.put((rank, {"losses": losses, "digest": _grad_digest(tr)[0]}))
    tr.close()
    _hold(tmp, port)


@pytest.mark.gpu
def test_zero1_bf16_wire_native_engine_side_stream(tmp_path):
    """ZeRO-1 with the bf16 wire on the native RCCL engine, weight gradients on the side stream
    (the staging buffers are allocated there and read on the engine's stream), three steps so freed
    staging blocks get reused: the same losses and gradients as torch.distributed's path."""
    nat = _run_ranks(_zero_wire_worker, 2, tmp_path, "native", timeout=120)
    tor = _run_ranks(_zero_wire_worker, 2, tmp_path, "torch", timeout=120)
    for r in (0, 1):
        assert all(math.isfinite(x) for x in nat[r]["losses"])
        assert nat[r]["losses"] == pytest.approx(tor[r]["losses"], rel=1e-5, abs=1e-5)
        torch.testing.assert_close(nat[r]["digest"], tor[r]["digest"], atol=1e-6, rtol=1e-3)


def test_rccl_channel_parse_reads_ring_lines_only(tmp_path):
    """bench.py's channel report takes the ring / tree layout lines of RCCL's INIT log, not the per-peer
    transport lines (whose number after the slash is a connection index)."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    log = tmp_path / "rccl.log"
    log.write_text(
        "host:1:1 [0] NCCL INFO Channel 00/04 :    0   1\n"
        "host:1:1 [0] NCCL INFO Channel 03/04 :    0   1\n"
        "host:1:1 [0] NCCL INFO Channel 00/0 : 0[0] -> 1[1] via P2P/IPC\n"
        "host:1:1 [0] NCCL INFO Channel 01/0 : 0[0] -> 1[1] via P2P/IPC comm 0x1\n"
        "host:1:1 [0] NCCL INFO Channel 00/16 :    0   1   2   3   4   5   6   7\n")
    assert bench._rccl_channels(str(log)) == [4, 16]
    assert bench._rccl_channels(str(tmp_path / "missing.log")) is None
