"""Worker-side failure detection and fault injection.

The reference has neither: a worker that dies is restarted by the training operator up to
``backoffLimit`` (``/root/reference/app/jobs/kubeflow/PyTorchJobDeployer.py:183``), and a worker that
*hangs* -- a lost peer leaves every other rank blocked in a collective -- holds its GPUs until someone
cancels the job.  Here:

* **Collective timeout** (``FTC_COLLECTIVE_TIMEOUT_S``, ``parallel.dist.init_distributed``): the
  process group's timeout.  RCCL's watchdog aborts a rank whose collective exceeds it (gloo raises),
  so the ranks still alive fail fast instead of waiting out torch's 30-minute default.
* **Step watchdog** (:class:`StepWatchdog`, ``FTC_STEP_TIMEOUT_S``): a host thread that ends the
  process with exit code 124 (the ``timeout(1)`` convention) when no optimizer step, evaluation or
  checkpoint write has completed for that long -- the case a collective timeout cannot see (a rank
  stuck *outside* collectives: data loader, a wedged kernel).  It dumps every thread's Python stack
  first, so the pod log names where the rank was stuck.
* **Fault injection** (:class:`FaultInjector`, ``FTC_FAULT``): ``<kind>@<step>[:rank=<r>]`` fires
  once per job at the start of optimizer step ``<step>`` (0-based) on rank ``<r>`` (default 0):

  ``crash``  raise -- a Python traceback, exit 1;
  ``oom``    SIGKILL itself -- what the kernel's OOM killer does (exit 137);
  ``hang``   block forever outside any collective -- to its peers, a lost RCCL rank.

  "Once per job" is a marker file in the checkpoint directory (which survives container restarts),
  so the restarted worker resumes from its checkpoint and runs through.  FakeCluster's
  ``inject_fault`` sets the variable on a job's pods; tests drive the whole restart path with it.
"""
from __future__ import annotations

import faulthandler
import logging
import os
import re
import signal
import sys
import threading
import time
from dataclasses import dataclass

log = logging.getLogger("ftc.faults")

KINDS = ("crash", "oom", "hang")
WATCHDOG_EXIT = 124


@dataclass(frozen=True)
class FaultSpec:
    kind: str
    step: int
    rank: int = 0

    @classmethod
    def parse(cls, text: str | None) -> "FaultSpec | None":
        if not text:
            return None
        m = re.fullmatch(r"\s*(\w+)@(\d+)(?::rank=(\d+))?\s*", text)
        if not m or m.group(1) not in KINDS:
            raise ValueError(f"FTC_FAULT={text!r}: expected <{'|'.join(KINDS)}>@<step>[:rank=<r>]")
        return cls(m.group(1), int(m.group(2)), int(m.group(3) or 0))

    @property
    def marker(self) -> str:
        return f".ftc_fault_{self.kind}_step{self.step}_rank{self.rank}"


class FaultInjector:
    def __init__(self, spec: FaultSpec | None, rank: int, state_dir: str):
        self.spec = spec if spec is not None and spec.rank == rank else None
        self.rank = rank
        self.state_dir = state_dir

    @classmethod
    def from_env(cls, rank: int, state_dir: str) -> "FaultInjector":
        return cls(FaultSpec.parse(os.environ.get("FTC_FAULT")), rank, state_dir)

    @property
    def armed(self) -> bool:
        return self.spec is not None and not os.path.exists(os.path.join(self.state_dir, self.spec.marker))

    def maybe_fire(self, step: int):
        if self.spec is None or step != self.spec.step or not self.armed:
            return
        path = os.path.join(self.state_dir, self.spec.marker)
        os.makedirs(self.state_dir, exist_ok=True)
        with open(path, "w") as f:  # durable before the fault: the restarted worker must not re-fire it
            f.write(f"{self.spec.kind} fired at step {step} on rank {self.rank} ({time.time():.0f})\n")
            f.flush()
            os.fsync(f.fileno())
        msg = f"[fault] injected {self.spec.kind} at step {step} on rank {self.rank}"
        print(msg, file=sys.stderr, flush=True)
        if self.spec.kind == "crash":
            raise RuntimeError(msg)
        if self.spec.kind == "oom":
            os.kill(os.getpid(), signal.SIGKILL)
        while True:  # hang: outside every collective; peers time out, the step watchdog ends this rank
            time.sleep(3600)


class StepWatchdog:
    """Exit(124) when :meth:`beat` has not been called for ``timeout_s`` seconds (0 = disabled)."""

    def __init__(self, timeout_s: float, rank: int = 0, exit_fn=None, poll_s: float | None = None,
                 first_timeout_s: float | None = None):
        self.timeout_s = float(timeout_s)
        # the first step also builds kernels' heuristics / TunableOp tables and warms allocators: until
        # the first beat the limit is max(3 x timeout, 300 s) unless given
        self.first_timeout_s = float(first_timeout_s) if first_timeout_s is not None else max(3 * self.timeout_s, 300.0)
        self._beats = 0
        self._phase_s = None  # one-off limit of the current phase (set by phase(), cleared by beat())
        self.rank = rank
        self._exit = exit_fn or os._exit
        self._last = time.monotonic()
        self._what = "start"
        self._stop = threading.Event()
        self._thread = None
        if self.timeout_s > 0:
            self._poll = poll_s if poll_s is not None else min(5.0, max(0.05, self.timeout_s / 10))
            self._thread = threading.Thread(target=self._run, name="ftc-step-watchdog", daemon=True)
            self._thread.start()

    @classmethod
    def from_env(cls, default_s: float, rank: int = 0) -> "StepWatchdog":
        return cls(float(os.environ.get("FTC_STEP_TIMEOUT_S", default_s) or 0), rank)

    def beat(self, what: str = ""):
        self._beats += 1
        self._phase_s = None
        self._last = time.monotonic()
        self._what = what or self._what

    def phase(self, what: str, timeout_s: float):
        """Start a phase with its own limit (the final save, the closing barrier): a rank whose peer died
        there still exits instead of hanging in a collective until the process-group timeout."""
        self._last = time.monotonic()
        self._what = what
        self._phase_s = float(timeout_s)

    def close(self):
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=1.0)

    def _run(self):
        while not self._stop.wait(self._poll):
            idle = time.monotonic() - self._last
            limit = self._phase_s if self._phase_s is not None else (self.timeout_s if self._beats else self.first_timeout_s)
            if idle > limit:
                print(f"[watchdog] rank {self.rank}: no progress for {idle:.0f} s (last: {self._what}); "
                      f"dumping stacks and exiting {WATCHDOG_EXIT}", file=sys.stderr, flush=True)
                try:
                    faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
                    sys.stderr.flush()
                finally:
                    self._exit(WATCHDOG_EXIT)
                return
