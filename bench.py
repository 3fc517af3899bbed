#!/usr/bin/env python3
"""Headline benchmark: fine-tune tokens/sec for the whole node, Llama-3-8B LoRA (BASELINE.json).

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One process per GPU (RCCL over xGMI for N > 1).  Each rank trains the FULL Llama-3-8B architecture
(random-init bf16 weights, synthetic uniform token ids) with LoRA r=16 / alpha=32 on all seven
linear projections of every layer -- forward, backward, bucketed gradient all-reduce overlapped
with backward, global grad-norm clip and the AdamW update are all inside the timed region.
Weak scaling: the per-GPU micro-batch is fixed, so global batch = micro_batch x N.

Launch modes:
* under torchrun (``WORLD_SIZE`` set): this process is one rank; ``--gpus`` must equal ``WORLD_SIZE``;
* ``--gpus N > 1`` with no ``WORLD_SIZE``: this process is a pure launcher -- it never imports torch
  or touches HIP, starts N rank processes (``RANK/LOCAL_RANK/WORLD_SIZE/MASTER_ADDR=127.0.0.1/
  MASTER_PORT``) as children, forwards rank 0's JSON line and exits with the first failing rank's
  code (terminating the rest).

W untimed warmup steps, then K steps bracketed by barrier + device synchronize on both sides; the
elapsed time is the MAX over ranks; rank 0 prints one JSON line on stdout and flushes it right after
the timed region.  Only then (never inside it, never before the line) do the ranks measure the
all-reduce bus bandwidth of one DDP-sized bucket, a bucket-size and an RCCL channel sweep -- on fresh
process groups with a 60 s collective timeout, under a total budget (``--diag-budget``, 120 s) after
which the sweep is abandoned and the process exits 0 -- and rank 0 writes them as one JSON object
(``{"diagnostics": ...}``) on stderr.  The default group's timeout is lowered to 300 s
(``--collective-timeout``) so a hang inside the timed steps fails the run before a driver's limit.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

BASELINE_METRIC = "fine-tune tokens/sec (whole node), Llama-3-8B LoRA at 1/2/4/8 MI355X"
DIAG_TIMEOUT_S = 60  # collective timeout of every post-headline diagnostic process group


def _mark(op: str):
    import torch

    try:
        if op == "push":
            torch.cuda.nvtx.range_push("ftc_timed")
        else:
            torch.cuda.nvtx.range_pop()
    except Exception:  # no roctx in this build: profiles fall back to whole-run stats
        pass


def _free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int, argv: list[str], timeout_s: float | None = None) -> int:
    """Launcher mode: start ``n`` rank processes of this script and supervise them.

    The parent imports nothing that initialises HIP (not even torch) and never exec()s: each rank
    is a child ``python bench.py <same args>`` with the torchrun-style env.  Rank 0's JSON line is
    relayed to stdout; every other line any rank prints goes to stderr.
    If any rank exits non-zero the others are terminated and that code is returned."""
    import signal
    import subprocess
    import threading

    port = int(os.environ.get("FTC_BENCH_PORT") or _free_port())
    procs = []
    relay_done = threading.Event()
    seen_json = []

    def relay(stream):
        for line in iter(stream.readline, ""):
            # the result line goes to stdout; anything else rank 0's libraries print there (gloo's
            # connection banner, ...) is diagnostics
            out = sys.stdout if line.lstrip().startswith("{") else sys.stderr
            out.write(line)
            out.flush()
            if out is sys.stdout:
                seen_json.append(line)
        relay_done.set()

    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
        p = subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env,
                             stdout=subprocess.PIPE if r == 0 else sys.stderr, text=True)
        procs.append(p)
    t = threading.Thread(target=relay, args=(procs[0].stdout,), daemon=True)
    t.start()
    t0 = time.monotonic()
    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = bad[0]
                break
            if all(c == 0 for c in codes):
                break
            if timeout_s and time.monotonic() - t0 > timeout_s:
                print(f"[bench] launcher timeout after {timeout_s:.0f}s", file=sys.stderr)
                rc = 124
                break
            time.sleep(0.2)
    except KeyboardInterrupt:
        rc = 130
    if rc != 0:
        for p in procs:  # the exact children we started
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
        deadline = time.monotonic() + 15
        for p in procs:
            try:
                p.wait(timeout=max(0.1, deadline - time.monotonic()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        print(f"[bench] a rank failed (exit {rc}); ranks' codes: {[p.returncode for p in procs]}", file=sys.stderr)
    relay_done.wait(timeout=10)
    if rc == 0 and not seen_json:
        print("[bench] rank 0 printed no JSON line", file=sys.stderr)
        rc = 1
    return rc if rc >= 0 else 128 - rc  # a signal-killed child (-N) -> 128+N


def _parse(argv):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--method", default="lora", choices=["lora", "qlora", "full"])
    ap.add_argument("--batch-size", type=int, default=4)
    ap.add_argument("--seq-len", type=int, default=4096)
    ap.add_argument("--lora-r", type=int, default=16)
    ap.add_argument("--bucket-mb", type=float, default=64.0)
    ap.add_argument("--comm-engine", default="torch", choices=["torch", "native"])
    ap.add_argument("--comm-ab", action="store_true",
                    help="after the timed region, also time the native RCCL engine's bucket all-reduce")
    ap.add_argument("--grad-dtype", default="auto", choices=["auto", "fp32", "bf16"],
                    help="gradient buffer / reduction dtype (full FT; auto: fp32 when accumulating)")
    ap.add_argument("--grad-wire", default="auto", choices=["auto", "bf16"],
                    help="gradient reduction dtype on the wire (bf16 over an fp32 buffer: half the bytes)")
    ap.add_argument("--rccl-channels", type=int, default=0,
                    help="> 0: NCCL_MIN/MAX_NCHANNELS for RCCL's communicators (set before the first GPU call)")
    ap.add_argument("--grad-accum", type=int, default=1)
    ap.add_argument("--zero-stage", type=int, default=-1, choices=[-1, 0, 1],
                    help="1: ZeRO-1 -- AdamW state sharded over the data-parallel ranks (reduce-scatter + all-gather); "
                         "-1 (auto): ZeRO-1 for full fine-tuning on > 1 GPU")
    ap.add_argument("--sp", type=int, default=1,
                    help="Ulysses sequence parallelism: groups of SP ranks share each sequence (1/SP of the tokens "
                         "per rank); --seq-len is the FULL sequence length")
    ap.add_argument("--checkpoint-layers", action="store_true")
    ap.add_argument("--ce-chunk-rows", type=int, default=4096,
                    help="rows per lm_head + cross-entropy chunk (the only vocab-sized buffer)")
    ap.add_argument("--kernels", default=None, choices=["hip", "torch"],
                    help="torch = stock PyTorch-ROCm ops (the 'before' row)")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu: plumbing rehearsal over gloo (tests); the metric is only meaningful on cuda")
    ap.add_argument("--graph", action="store_true", help="whole training step captured in a hipGraph (1 GPU)")
    ap.add_argument("--doc-len", type=int, default=0,
                    help="packed documents of this many tokens (document-masked attention; 0: one per row)")
    ap.add_argument("--profile-steps", type=int, default=0, help="extra steps under torch.profiler (not timed)")
    ap.add_argument("--launcher-timeout", type=float, default=0.0,
                    help="launcher mode: give up after this many seconds (0: never)")
    ap.add_argument("--diag-budget", type=float, default=120.0,
                    help="N > 1: seconds for the post-headline transport diagnostics (bucket / size / channel "
                         "sweeps) before they are abandoned and the rank exits 0; 0 skips them")
    ap.add_argument("--collective-timeout", type=float, default=300.0,
                    help="process-group collective timeout (s): a hang inside the timed steps aborts the ranks "
                         "(non-zero exit) well before a driver's limit; FTC_COLLECTIVE_TIMEOUT_S overrides")
    return ap.parse_args(argv)


def _rccl_channels(path: str | None) -> list[int] | None:
    """Channel counts RCCL chose for this rank's communicators, from its INIT log lines
    (``Channel 00/16 : 0 1 ...`` -> 16); None when there is no log (1 rank, CPU, a user NCCL_DEBUG)."""
    import re

    if not path or not os.path.exists(path):
        return None
    # the ring / tree layout lines ("Channel 03/16 :    0   1") -- not the per-connection transport lines
    # ("Channel 00/0 : 0[0] -> 1[1] via P2P/IPC", whose number after the slash is a connection index)
    ring = re.compile(r"Channel \d+/(\d+) :(?:\s+\d+)+\s*$")
    found = set()
    with open(path, errors="replace") as f:
        for ln in f:
            m = ring.search(ln)
            if m:
                found.add(int(m.group(1)))
    return sorted(found)


def _channel_sweep(info, mb: float, counts=(2, 4, 8, 16)) -> dict:
    """Bus bandwidth of the ``mb``-MB bucket all-reduce on fresh RCCL communicators pinned to each channel
    count (ncclConfig_t min/maxCTAs through ProcessGroupNCCL.Options): tells channel starvation from link
    bandwidth in the first 8-GPU record.  Errors are reported, never raised."""
    import datetime

    import torch.distributed as dist

    out = {}
    for c in counts:
        try:
            opts = dist.ProcessGroupNCCL.Options()
            opts.config.min_ctas = c
            opts.config.max_ctas = c
            opts._timeout = datetime.timedelta(seconds=DIAG_TIMEOUT_S)  # the same as the kwarg: no override warning
            g = dist.new_group(backend="nccl", pg_options=opts, timeout=datetime.timedelta(seconds=DIAG_TIMEOUT_S))
            out[str(c)] = _bucket_busbw(info, mb, iters=5, group=g)["busbw_GBps"]
            dist.destroy_process_group(g)
        except Exception as e:  # noqa: BLE001 -- a diagnostic
            out[str(c)] = f"error: {type(e).__name__}: {e}"[:160]
    return out


def _bucket_busbw(info, mb: float, native=None, iters: int = 10, group=None) -> dict:
    """Bus bandwidth (GB/s) of one ``mb``-MB bf16 SUM all-reduce, the DDP bucket size: algbw x
    2(n-1)/n, the per-link rate a ring moves (nccl-tests convention)."""
    import torch
    import torch.distributed as dist

    from finetune_controller_amd.parallel import dist as pdist

    n = info.world_size
    numel = int(mb * 2 ** 20 / 2)
    t = torch.ones(numel, device=info.device, dtype=torch.bfloat16)
    cuda = info.device.type == "cuda"

    def run():
        if native is not None:
            native.all_reduce_async(t).wait()
        else:
            dist.all_reduce(t, group=group)

    for _ in range(3):
        run()
    if native is not None:
        native.reset()
    if cuda:
        torch.cuda.synchronize(info.device)
    if group is None:
        pdist.barrier(info)
    else:  # a diagnostic group: its own (short) timeout, not the default group's
        dist.all_reduce(torch.zeros(1, device=info.device), group=group)
        if cuda:
            torch.cuda.synchronize(info.device)
    t0 = time.perf_counter()
    for _ in range(iters):
        run()
    if cuda:
        torch.cuda.synchronize(info.device)
    sec = (time.perf_counter() - t0) / iters
    if native is not None:
        native.reset()
    sec = max(sec, 1e-9)
    return {"bucket_mb": mb, "ms": round(sec * 1e3, 3),
            "busbw_GBps": round(numel * 2 / sec / 1e9 * 2 * (n - 1) / n, 1)}


def _run_diagnostics(a, info, tr, dev, cuda: bool, budget_s: float) -> dict:
    """Post-headline transport diagnostics in a daemon thread, joined for at most ``budget_s``.

    Every collective runs on a fresh process group whose timeout is ``DIAG_TIMEOUT_S``.  Returns the
    results; ``abandoned`` is set when the budget ran out (the caller then exits 0 without joining).
    Fault hook for the tests: ``FTC_BENCH_DIAG_STALL_RANK=<r>`` parks rank r inside the sweep."""
    import datetime
    import threading

    import torch
    import torch.distributed as dist

    res: dict = {"budget_s": budget_s, "group_timeout_s": DIAG_TIMEOUT_S}
    done = threading.Event()
    t0 = time.monotonic()

    def work():
        try:
            if cuda:
                torch.cuda.set_device(dev)  # the current device is per thread
            g = dist.new_group(backend=info.backend, timeout=datetime.timedelta(seconds=DIAG_TIMEOUT_S))
            stall = os.environ.get("FTC_BENCH_DIAG_STALL_RANK")
            if stall not in (None, "") and int(stall) == info.rank:
                time.sleep(10 ** 6)
            res["torch"] = _bucket_busbw(info, a.bucket_mb, group=g)
            if cuda:  # bucket-size sweep: xGMI data for tuning bucket_mb
                res["sweep_busbw_GBps"] = {str(mb): _bucket_busbw(info, mb, iters=5, group=g)["busbw_GBps"]
                                           for mb in (4, 16, 64, 256)}
                res["channel_sweep_busbw_GBps"] = _channel_sweep(info, a.bucket_mb)
            if cuda and (a.comm_ab or a.comm_engine == "native"):
                try:
                    native = tr.ddp._native
                    if native is None:
                        from finetune_controller_amd.parallel.comm import NativeComm

                        native = NativeComm(device=dev)
                    res["native"] = _bucket_busbw(info, a.bucket_mb, native=native, group=g)
                except Exception as e:  # noqa: BLE001 -- a diagnostic
                    res["native"] = {"error": f"{type(e).__name__}: {e}"[:200]}
        except Exception as e:  # noqa: BLE001 -- report, never fail the run on a diagnostic
            res["error"] = f"{type(e).__name__}: {e}"[:300]
        finally:
            done.set()

    threading.Thread(target=work, name="ftc-bench-diag", daemon=True).start()
    if not done.wait(budget_s):
        res["abandoned"] = True
    res["elapsed_s"] = round(time.monotonic() - t0, 2)
    return res


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    a = _parse(argv)
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and a.gpus > 1:
        return spawn_ranks(a.gpus, argv, a.launcher_timeout or None)
    if world_env is not None and int(world_env) != a.gpus:
        print(f"[bench] --gpus {a.gpus} but WORLD_SIZE={world_env}: refusing to report a mislabelled number",
              file=sys.stderr)
        return 2
    if a.kernels:
        os.environ["FTC_KERNELS"] = a.kernels
    # RCCL's intra-node buffers travel by dmabuf IPC on these hosts; the legacy IPC handle path fails
    # (hipIpcGetMemHandle: invalid argument).  Read by the HIP runtime at its first call, i.e. after here.
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    # RCCL reads these at communicator creation, i.e. after here
    if a.rccl_channels > 0:
        os.environ["NCCL_MIN_NCHANNELS"] = os.environ["NCCL_MAX_NCHANNELS"] = str(a.rccl_channels)
    rccl_log = None
    if (a.device == "cuda" and a.gpus > 1 and "NCCL_DEBUG_FILE" not in os.environ
            and os.environ.get("NCCL_DEBUG", "").upper() in ("", "VERSION", "WARN", "NONE")):
        # the channel count RCCL picks is in its INIT log lines: to a per-rank file (never stdout); a
        # launcher's NCCL_DEBUG=VERSION / WARN is raised to INIT-subsystem INFO for this file only
        import tempfile

        rccl_log = os.path.join(tempfile.gettempdir(), f"ftc_rccl_{os.getpid()}.log")
        os.environ.update(NCCL_DEBUG="INFO", NCCL_DEBUG_SUBSYS="INIT", NCCL_DEBUG_FILE=rccl_log)

    # the default process group's collective timeout (read by parallel.dist.init_distributed): a hang in
    # the timed steps ends the ranks with a non-zero code long before a driver's limit (torch: 1800 s)
    os.environ.setdefault("FTC_COLLECTIVE_TIMEOUT_S", str(int(a.collective_timeout)))
    pg_timeout_s = int(float(os.environ["FTC_COLLECTIVE_TIMEOUT_S"]))

    import torch
    import torch.distributed as dist

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from finetune_controller_amd.parallel import dist as pdist
    from finetune_controller_amd.train.trainer import TrainConfig, Trainer

    cuda = a.device == "cuda"
    tc = TrainConfig(model=a.model, method=a.method, lora_r=a.lora_r, lora_alpha=2.0 * a.lora_r,
                     batch_size=a.batch_size, seq_len=a.seq_len, synthetic=True, max_steps=a.warmup + a.steps,
                     warmup_steps=0, schedule="constant", lr=1e-4, bucket_mb=a.bucket_mb, comm_engine=a.comm_engine,
                     zero_stage=a.zero_stage, grad_accum=a.grad_accum, grad_dtype=a.grad_dtype,
                     grad_wire=a.grad_wire, sp=a.sp,
                     checkpoint_layers=a.checkpoint_layers, ce_chunk_rows=a.ce_chunk_rows, save_model=False,
                     resume=False, device=a.device, pack_documents=a.doc_len > 0, eos_id=2,
                     synthetic_doc_len=a.doc_len, graph=a.graph, comm_probe=a.gpus > 1)
    tr = Trainer(tc)
    info = tr.info
    dev = tr.device

    def sync():
        if cuda:
            torch.cuda.synchronize(dev)

    for _ in range(a.warmup):
        tr.train_step(tc.lr)
    sync()
    pdist.barrier(info)
    sync()
    tr.comm_exposed_ms()  # drop the warm-up steps' probes (events only: nothing synchronises in the loop)
    tr.param_sync_exposed_ms()
    if cuda:
        _mark("push")  # roctx range "ftc_timed" (rocprofv3 --marker-trace; tools/kstats_md.py filters on it)
    t0 = time.perf_counter()
    last = None
    for _ in range(a.steps):
        last = tr.train_step(tc.lr)
    sync()
    pdist.barrier(info)
    sync()
    elapsed_rank = time.perf_counter() - t0
    if cuda:
        _mark("pop")
    elapsed = pdist.all_reduce_max(elapsed_rank, info)
    fastest = -pdist.all_reduce_max(-elapsed_rank, info)
    # gradient-reduction time backward did not hide, measured by device events inside the timed steps
    exposed = tr.comm_exposed_ms()
    exposed = pdist.all_reduce_max(exposed, info) if exposed is not None else None
    # ZeRO-1: the parameter all-gather time the update / next forward did not hide
    psync = tr.param_sync_exposed_ms()
    psync = pdist.all_reduce_max(psync, info) if psync is not None else None
    loss = float(last.float().item()) if last is not None else float("nan")

    n = info.world_size
    pg_world = dist.get_world_size() if dist.is_initialized() else 1
    ngroups = n // max(1, a.sp)  # data-parallel replicas; an SP group trains B full sequences together
    tokens = a.batch_size * a.seq_len * a.grad_accum * ngroups * a.steps
    value = tokens / elapsed
    ms = elapsed / a.steps * 1000
    flops_tok = tr.cfg.flops_per_token(a.seq_len, lora=a.method != "full")

    channels = _rccl_channels(rccl_log) if info.is_main else None  # before any diagnostic communicator
    rccl = None
    if cuda:
        try:
            v = torch.cuda.nccl.version()
            rccl = ".".join(str(x) for x in v) if isinstance(v, tuple) else str(v)
        except Exception:
            rccl = None
    # peer access from this rank's GPU (xGMI P2P: RCCL's direct transport on an 8-GPU node; a rehearsal
    # on one shared card reports none) -- makes the first multi-GPU record self-describing
    p2p = None
    if cuda and n > 1:
        try:
            me = dev.index if dev.index is not None else torch.cuda.current_device()
            p2p = sum(1 for j in range(torch.cuda.device_count()) if j != me and torch.cuda.can_device_access_peer(me, j))
        except Exception:
            p2p = None

    # ---- the headline line FIRST: printed and flushed before any post-timed collective, so a diagnostic
    # that stalls on a first real xGMI node can never cost the record
    if info.is_main:
        from finetune_controller_amd.ops import _backend

        out = {
            # the BASELINE.json metric names the headline config; any other model / method says what it is
            "metric": BASELINE_METRIC if (a.model, a.method) == ("llama3-8b", "lora")
            else f"fine-tune tokens/sec (whole node), {a.model} {a.method}",
            "value": round(value, 1),
            "unit": "tokens/s",
            "n_gpus": n,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16" if cuda else "fp32",
            "data": "synthetic (uniform random token ids; random-init weights)",
            "config": {
                "model": a.model,
                "method": a.method,
                "lora": {"r": a.lora_r, "alpha": 2 * a.lora_r, "targets": "all-linear"} if a.method != "full" else None,
                "global_batch": a.batch_size * a.grad_accum * ngroups,
                "micro_batch_per_gpu": a.batch_size,
                "grad_accum": a.grad_accum,
                "seq_len": a.seq_len,
                "tokens_per_step": a.batch_size * a.seq_len * a.grad_accum * ngroups,
                "parallelism": f"dp{ngroups}" + (f"-sp{a.sp}" if a.sp > 1 else "")
                               + ("-zero1" if tr.zero_stage and n > 1 else ""),
                "kernels": _backend.kernel_mode(),
                "comm_engine": a.comm_engine,
                "zero_stage": tr.zero_stage,
                "grad_dtype": str(tr.opt.grad_flat.dtype).replace("torch.", ""),
                "device": a.device,
                **({"packed_doc_len": a.doc_len} if a.doc_len else {}),
                **({"hipgraph": True} if tr.graph_ok() else {}),
            },
            "world_size_pg": pg_world,
            "dist_backend": info.backend,
            "rccl_version": rccl,
            "rccl_channels": channels,
            "p2p_peers": p2p,
            "rank_ms_per_step": {"max": round(ms, 2), "min": round(fastest / a.steps * 1000, 2)},
            "comm": {
                "comm_exposed_ms": None if exposed is None else round(exposed, 3),
                "param_sync_exposed_ms": None if psync is None else round(psync, 3),
                "zero_gather_overlap": bool(tr.zero_stage and getattr(tr.opt, "_stage_buckets", None) is not None),
                "wire_GB_per_step": round(tr.ddp.wire_bytes_per_step() / 1e9, 6),
                "n_buckets": tr.ddp.n_collectives(),
                "bucket_mb": a.bucket_mb,
                "grad_wire": str(tr.ddp.wire_dtype or tr.opt.grad_flat.dtype).replace("torch.", ""),
                "collective_timeout_s": pg_timeout_s,
                "env": {k: v for k, v in sorted(os.environ.items())
                        if k.startswith(("NCCL_", "RCCL_")) or k in ("HSA_ENABLE_IPC_MODE_LEGACY", "FTC_SHARE_GPU")},
            },
            "loss": round(loss, 4),
            "model_tflops_per_gpu": round(value * flops_tok / n / 1e12, 1),
            "peak_mem_gb": round(torch.cuda.max_memory_allocated(dev) / 1e9, 1) if cuda else None,
        }
        print(json.dumps(out), flush=True)
    sys.stderr.flush()

    # ---- after the headline: transport diagnostics (never part of the metric), on their own process
    # groups with a short collective timeout, in a worker thread under a total budget.  Past the budget
    # the sweep is abandoned and the rank exits 0 at once (the headline is already out); a stalled RCCL
    # kernel of an abandoned sweep dies with the process.
    if n > 1 and a.diag_budget > 0:
        diag = _run_diagnostics(a, info, tr, dev, cuda, budget_s=a.diag_budget)
        if info.is_main:
            print(json.dumps({"diagnostics": diag}), file=sys.stderr, flush=True)
        if diag.get("abandoned"):
            sys.stdout.flush()
            sys.stderr.flush()
            if rccl_log and os.path.exists(rccl_log):
                os.remove(rccl_log)
            os._exit(0)

    if a.profile_steps:
        from torch.profiler import ProfilerActivity, profile

        acts = [ProfilerActivity.CPU] + ([ProfilerActivity.CUDA] if cuda else [])
        with profile(activities=acts) as prof:
            for _ in range(a.profile_steps):
                tr.train_step(tc.lr)
            sync()
        if info.is_main:
            os.makedirs("gpurun_out", exist_ok=True)
            with open("gpurun_out/torch_profile.txt", "w") as f:
                f.write(prof.key_averages().table(sort_by="cuda_time_total" if cuda else "cpu_time_total",
                                                  row_limit=60))
    tr.close()
    if rccl_log and os.path.exists(rccl_log):  # this rank's RCCL INIT log: parsed above, not kept
        os.remove(rccl_log)
    return 0


if __name__ == "__main__":
    sys.exit(main())
