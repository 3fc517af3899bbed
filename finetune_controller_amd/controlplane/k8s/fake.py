"""FakeCluster: an in-process Kubernetes with the Kubeflow training operator and Kueue emulated.

The reference can only be exercised against a real OpenShift cluster.  This fake
implements the ``KubeClient`` protocol and reconciles exactly the state the control plane reads:

* **Kueue** -- a ``Workload`` per suspended PyTorchJob whose queue label names a LocalQueue; the
  Workload carries ``QuotaReserved=False`` until its ClusterQueue has room for the job's aggregate
  requests (cpu / memory / ``amd.com/gpu`` ...), admission is FIFO by creationTimestamp (the ordering
  ``get_kueue_queue`` reconstructs, ``/root/reference/app/utils/kueue_helpers.py:19-46``); admitting
  sets ``QuotaReserved=True`` and clears ``runPolicy.suspend``; finished jobs release quota.
* **training operator** -- conditions ``Created`` -> (``Suspended``) -> ``Running`` -> ``Succeeded`` /
  ``Failed`` with ``Restarting`` in between retries (``backoffLimit``), ``startTime`` /
  ``completionTime``, ``replicaStatuses.Master.selector`` and pods labelled
  ``training.kubeflow.org/job-name`` / ``replica-type``.
* **pods** -- either really executed (``run_processes``: the ``pytorch`` container's command runs as a
  local subprocess with ``/data/dataset`` and ``/data/artifacts`` mapped to temp dirs, the dataset
  init container and the ``s3-sync`` sidecar emulated against an ``ObjectStore``), or simulated (a
  scripted log + ``metrics.csv`` and success after ``sim_ticks`` reconcile ticks).  By default jobs
  that request no GPU run for real and GPU jobs are simulated.
* **fault injection** -- ``kill_pod`` (process killed -> restart path), ``fail_next`` (scripted failure),
  ``oom`` (exit 137).
"""
from __future__ import annotations

import copy
import datetime as _dt
import fnmatch
import os
import re
import shlex
import signal
import subprocess
import sys
import tempfile
import threading
import time
import uuid

from .client import JOB_NAME_LABEL, JOB_ROLE_LABEL, REPLICA_TYPE_LABEL, KubeClient, KubeError
from .manifest import QUEUE_LABEL, total_requests
from .quantity import parse_quantity

REPO_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def _now() -> str:
    return _dt.datetime.now(_dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")


def _match_selector(labels: dict, selector: str | None) -> bool:
    if not selector:
        return True
    for part in selector.split(","):
        k, _, v = part.partition("=")
        if labels.get(k.strip()) != v.strip():
            return False
    return True


class _Pod:
    def __init__(self, name, job, rtype, index, spec, labels):
        self.name, self.job, self.rtype, self.index = name, job, rtype, index
        self.spec, self.labels = spec, labels
        self.phase = "Pending"
        self.logs: list[str] = []
        self.proc: subprocess.Popen | None = None
        self.exit_code: int | None = None
        self.restarts = 0
        self.start_time = None
        self.finish_time = None
        self.workdir = None
        self.sim_left = 0
        self.lock = threading.Lock()
        self.sync_thread = None
        self.log_cond = threading.Condition()

    def append_log(self, line: str):
        with self.log_cond:
            self.logs.append(line.rstrip("\n"))
            self.log_cond.notify_all()

    def as_dict(self, namespace):
        cs = [{"name": "pytorch", "restartCount": self.restarts, "ready": self.phase == "Running",
               "state": ({"terminated": {"exitCode": self.exit_code, "finishedAt": self.finish_time}}
                         if self.exit_code is not None else
                         ({"running": {"startedAt": self.start_time}} if self.phase == "Running" else
                          {"waiting": {"reason": "ContainerCreating", "message": "pulling image"}}))}]
        return {"metadata": {"name": self.name, "namespace": namespace, "labels": dict(self.labels)},
                "spec": self.spec,
                "status": {"phase": self.phase, "startTime": self.start_time, "containerStatuses": cs}}


def kueue_quotas_from_manifests(docs) -> tuple[dict, dict]:
    """(cluster_queues, local_queues) for FakeCluster from Kueue ClusterQueue / LocalQueue manifests.

    The fake admits by per-ClusterQueue totals: each resource's nominalQuota is summed over the
    queue's flavors (flavor placement, cohort borrowing and preemption are not simulated)."""
    cqs, lqs = {}, {}
    for d in docs:
        if not d:
            continue
        if d.get("kind") == "ClusterQueue":
            tot: dict = {}
            for group in d["spec"].get("resourceGroups", []):
                for fl in group.get("flavors", []):
                    for r in fl.get("resources", []):
                        tot[r["name"]] = tot.get(r["name"], 0.0) + parse_quantity(r["nominalQuota"])
            cqs[d["metadata"]["name"]] = tot
        elif d.get("kind") == "LocalQueue":
            lqs[d["metadata"]["name"]] = d["spec"]["clusterQueue"]
    return cqs, lqs


class FakeCluster(KubeClient):
    def __init__(self, object_store=None, run_processes: bool | str = "cpu", workdir: str | None = None,
                 cluster_queues: dict | None = None, local_queues: dict | None = None, sim_ticks: int = 3,
                 sync_interval: float = 0.5, secrets: dict | None = None, python: str | None = None):
        self.store = object_store
        self.run_processes = run_processes  # True | False | "cpu" (only jobs without GPU requests)
        self.workdir = workdir or tempfile.mkdtemp(prefix="ftc-fakecluster-")
        self.cluster_queues = cluster_queues if cluster_queues is not None else {
            "cluster-queue": {"cpu": 64, "memory": "512Gi", "amd.com/gpu": 8}}
        self.local_queues = local_queues if local_queues is not None else {
            "finetune-queue": "cluster-queue", "user-queue": "cluster-queue"}
        self.sim_ticks = sim_ticks
        self.sync_interval = sync_interval
        self.secrets = secrets or {}
        self.python = python or sys.executable
        self.objects: dict[tuple, dict] = {}
        self.pods: dict[tuple, _Pod] = {}
        self.events: list[dict] = []
        self.usage: dict[str, dict[str, float]] = {cq: {} for cq in self.cluster_queues}
        self.admitted: dict[tuple, tuple[str, dict]] = {}
        self.lock = threading.RLock()
        self._thread = None
        self._stop = threading.Event()
        self._fail_next: set[str] = set()
        self._fault_env: dict[str, dict[str, str]] = {}
        self.history: list[tuple[str, str]] = []  # (job, condition) transitions, for tests
        self.deleted_pod_logs: dict[str, list[str]] = {}  # logs of pods removed with their job

    # ------------------------------------------------------------------ KubeClient API

    def set_kueue(self, cluster_queues: dict, local_queues: dict):
        """Replace the queue topology (e.g. from ``kueue_quotas_from_manifests``) before any admission."""
        self.cluster_queues, self.local_queues = cluster_queues, local_queues
        self.usage = {cq: {} for cq in cluster_queues}
    def create_custom(self, group, version, namespace, plural, body):
        with self.lock:
            name = body["metadata"]["name"]
            key = (group, plural, namespace, name)
            if key in self.objects:
                raise KubeError(409, "AlreadyExists", name)
            obj = copy.deepcopy(body)
            md = obj.setdefault("metadata", {})
            md.setdefault("namespace", namespace)
            md["uid"] = str(uuid.uuid4())
            md["creationTimestamp"] = _now()
            md["_seq"] = len(self.objects)
            self.objects[key] = obj
            if plural == "pytorchjobs":
                obj["status"] = {"conditions": []}
                self._set_condition(obj, "Created", "PyTorchJobCreated", f"PyTorchJob {name} is created.")
                if obj["spec"]["runPolicy"].get("suspend"):
                    self._set_condition(obj, "Suspended", "PyTorchJobSuspended", f"PyTorchJob {name} is suspended.")
            self._event(namespace, name, "Normal", "Created", f"{plural}/{name} created")
            return copy.deepcopy(obj)

    def get_custom(self, group, version, namespace, plural, name):
        with self.lock:
            obj = self.objects.get((group, plural, namespace, name))
            if obj is None:
                raise KubeError(404, "NotFound", name)
            return copy.deepcopy(obj)

    def delete_custom(self, group, version, namespace, plural, name):
        with self.lock:
            key = (group, plural, namespace, name)
            obj = self.objects.pop(key, None)
            if obj is None:
                raise KubeError(404, "NotFound", name)
            if plural == "pytorchjobs":
                self._release(namespace, name)
                self.objects.pop(("kueue.x-k8s.io", "workloads", namespace, f"pytorchjob-{name}"), None)
                for pkey in [k for k in self.pods if k[0] == namespace and self.pods[k].job == name]:
                    pod = self.pods.pop(pkey)
                    self.deleted_pod_logs[pod.name] = list(pod.logs)
                    self._kill(pod)
            return {"status": "Success", "metadata": obj["metadata"]}

    def list_custom(self, group, version, namespace, plural, label_selector=None):
        with self.lock:
            items = [copy.deepcopy(o) for (g, p, ns, _), o in self.objects.items()
                     if g == group and p == plural and ns == namespace
                     and _match_selector(o["metadata"].get("labels", {}), label_selector)]
            items.sort(key=lambda o: o["metadata"]["_seq"])
            return {"items": items}

    def list_pods(self, namespace, label_selector=None):
        with self.lock:
            return [p.as_dict(namespace) for (ns, _), p in self.pods.items()
                    if ns == namespace and _match_selector(p.labels, label_selector)]

    def read_pod(self, namespace, name):
        with self.lock:
            p = self.pods.get((namespace, name))
            if p is None:
                raise KubeError(404, "NotFound", name)
            return p.as_dict(namespace)

    def read_pod_log(self, namespace, name, container=None, tail_lines=None):
        p = self.pods.get((namespace, name))
        if p is None:
            raise KubeError(404, "NotFound", name)
        with p.log_cond:
            lines = list(p.logs)
        if tail_lines:
            lines = lines[-int(tail_lines):]
        return "\n".join(lines) + ("\n" if lines else "")

    def stream_pod_log(self, namespace, name, container=None, tail_lines=None):
        p = self.pods.get((namespace, name))
        if p is None:
            raise KubeError(404, "NotFound", name)
        with p.log_cond:
            i = max(0, len(p.logs) - int(tail_lines)) if tail_lines else 0
        while True:
            with p.log_cond:
                while i >= len(p.logs) and p.phase in ("Pending", "Running"):
                    p.log_cond.wait(timeout=0.2)
                    if self._stop.is_set():
                        return
                if i < len(p.logs):
                    line = p.logs[i]
                    i += 1
                else:
                    return  # pod finished and drained
            yield (line + "\n").encode()

    def list_events(self, namespace):
        with self.lock:
            return [copy.deepcopy(e) for e in self.events if e["metadata"]["namespace"] == namespace]

    def read_secret(self, name, namespace):
        if name not in self.secrets:
            raise KubeError(404, "NotFound", name)
        return dict(self.secrets[name])

    # ------------------------------------------------------------------ fault injection
    def kill_pod(self, namespace, job_name, exit_code: int = 137):
        with self.lock:
            for p in self.pods.values():
                if p.job == job_name and p.rtype == "master":
                    if p.proc and p.proc.poll() is None:
                        p.proc.send_signal(signal.SIGKILL)
                    else:
                        p.exit_code = exit_code
                        p.sim_left = 0

    def fail_next(self, job_name: str):
        self._fail_next.add(job_name)

    def inject_fault(self, job_name: str, fault: str | None = None, collective_timeout_s: float | None = None,
                     step_timeout_s: float | None = None):
        """Worker-side faults for a job's processes (``utils.faults``): ``fault`` is an ``FTC_FAULT``
        spec -- ``crash@3``, ``oom@2:rank=1``, ``hang@2:rank=1`` (a lost RCCL peer) -- fired once per
        job; the timeouts are the worker's failure detectors (``FTC_COLLECTIVE_TIMEOUT_S``,
        ``FTC_STEP_TIMEOUT_S``).  Applies to every pod (re)started after the call."""
        env = self._fault_env.setdefault(job_name, {})
        if fault:
            env["FTC_FAULT"] = fault
        if collective_timeout_s is not None:
            env["FTC_COLLECTIVE_TIMEOUT_S"] = str(collective_timeout_s)
        if step_timeout_s is not None:
            env["FTC_STEP_TIMEOUT_S"] = str(step_timeout_s)

    # ------------------------------------------------------------------ reconciliation
    def start(self, tick: float = 0.2):
        if self._thread:
            return
        self._stop.clear()

        def loop():
            while not self._stop.is_set():
                try:
                    self.reconcile()
                except Exception as e:  # keep the simulator alive
                    print(f"[fakecluster] reconcile error: {e!r}", file=sys.stderr)
                self._stop.wait(tick)

        self._thread = threading.Thread(target=loop, name="fakecluster", daemon=True)
        self._thread.start()

    def stop(self):
        self._stop.set()
        if self._thread:
            self._thread.join(timeout=5)
            self._thread = None
        with self.lock:
            for p in self.pods.values():
                self._kill(p)

    def reconcile(self):
        with self.lock:
            jobs = [(k, o) for k, o in self.objects.items() if k[1] == "pytorchjobs"]
            jobs.sort(key=lambda kv: kv[1]["metadata"]["_seq"])
            for (g, pl, ns, name), job in jobs:
                self._reconcile_kueue(ns, name, job)
            for (g, pl, ns, name), job in jobs:
                self._reconcile_job(ns, name, job)

    # ---- Kueue ----
    def _reconcile_kueue(self, ns, name, job):
        lq = job["metadata"].get("labels", {}).get(QUEUE_LABEL)
        if not lq:
            return
        wkey = ("kueue.x-k8s.io", "workloads", ns, f"pytorchjob-{name}")
        wl = self.objects.get(wkey)
        if wl is None and job["spec"]["runPolicy"].get("suspend"):
            wl = {"apiVersion": "kueue.x-k8s.io/v1beta1", "kind": "Workload",
                  "metadata": {"name": wkey[3], "namespace": ns, "creationTimestamp": job["metadata"]["creationTimestamp"],
                               "_seq": job["metadata"]["_seq"],
                               "ownerReferences": [{"kind": "PyTorchJob", "name": name}],
                               "labels": {QUEUE_LABEL: lq}},
                  "spec": {"queueName": lq},
                  "status": {"conditions": [{"type": "QuotaReserved", "status": "False", "reason": "Pending",
                                             "message": "waiting for quota", "lastTransitionTime": _now()}]}}
            self.objects[wkey] = wl
        if wl is None or not self._pending(wl):
            return
        cq = self.local_queues.get(lq)
        if cq is None or cq not in self.cluster_queues:
            wl["status"]["conditions"][0]["message"] = f"LocalQueue {lq} doesn't exist"
            return
        # FIFO: only admit if every older pending workload of this ClusterQueue is admitted
        for (g, p, wns, wname), other in sorted(self.objects.items(), key=lambda kv: kv[1]["metadata"].get("_seq", 0)):
            if p != "workloads" or other is wl:
                continue
            if self.local_queues.get(other["spec"]["queueName"]) == cq and self._pending(other) and \
                    other["metadata"]["_seq"] < wl["metadata"]["_seq"]:
                return
        req = total_requests(job)
        quota = {k: parse_quantity(v) for k, v in self.cluster_queues[cq].items()}
        used = self.usage[cq]
        for res, amt in req.items():
            if amt <= 0:
                continue
            if res not in quota or used.get(res, 0.0) + amt > quota[res] + 1e-9:
                wl["status"]["conditions"][0]["message"] = f"insufficient quota for {res} in ClusterQueue {cq}"
                return
        for res, amt in req.items():
            used[res] = used.get(res, 0.0) + amt
        self.admitted[(ns, name)] = (cq, req)
        wl["status"]["conditions"] = [
            {"type": "QuotaReserved", "status": "True", "reason": "QuotaReserved",
             "message": f"Quota reserved in ClusterQueue {cq}", "lastTransitionTime": _now()},
            {"type": "Admitted", "status": "True", "reason": "Admitted", "message": "admitted",
             "lastTransitionTime": _now()}]
        job["spec"]["runPolicy"]["suspend"] = False
        self._event(ns, name, "Normal", "Admitted", f"workload admitted by ClusterQueue {cq}")

    @staticmethod
    def _pending(wl) -> bool:
        return any(c["type"] == "QuotaReserved" and c["status"] == "False" for c in wl["status"]["conditions"])

    def _release(self, ns, name):
        ad = self.admitted.pop((ns, name), None)
        if ad:
            cq, req = ad
            for res, amt in req.items():
                self.usage[cq][res] = self.usage[cq].get(res, 0.0) - amt

    # ---- operator ----
    def _reconcile_job(self, ns, name, job):
        st = job["status"]
        last = st["conditions"][-1]["type"] if st["conditions"] else None
        if last in ("Succeeded", "Failed"):
            return
        if job["spec"]["runPolicy"].get("suspend"):
            if last != "Suspended":
                self._set_condition(job, "Suspended", "PyTorchJobSuspended", f"PyTorchJob {name} is suspended.")
            return
        pods = [p for (pns, _), p in self.pods.items() if pns == ns and p.job == name]
        if not pods:
            pods = self._create_pods(ns, name, job)
            st.setdefault("startTime", _now())
            st["replicaStatuses"] = {"Master": {"active": 1, "selector":
                                                f"{JOB_NAME_LABEL}={name},{REPLICA_TYPE_LABEL}=master"}}
            if last != "Created":
                self._set_condition(job, "Created", "PyTorchJobCreated", f"PyTorchJob {name} is created.")
            return
        for p in pods:
            self._advance_pod(ns, job, p)
        if all(p.phase == "Running" for p in pods) and last not in ("Running",):
            self._set_condition(job, "Running", "PyTorchJobRunning", f"PyTorchJob {name} is running.")
            return
        failed = [p for p in pods if p.exit_code not in (None, 0)]
        if failed:
            backoff = int(job["spec"]["runPolicy"].get("backoffLimit", 0))
            p = failed[0]
            if p.restarts < backoff:
                p.restarts += 1
                self._set_condition(job, "Restarting", "PyTorchJobRestarting",
                                    f"PyTorchJob {name} is restarting because {p.name} exited with {p.exit_code}.")
                self._start_pod(ns, job, p)
                return
            st["completionTime"] = _now()
            self._set_condition(job, "Failed", "PyTorchJobFailed",
                                f"PyTorchJob {name} is failed because {p.name} exited with code {p.exit_code}.")
            self._release(ns, name)
            return
        if all(p.exit_code == 0 for p in pods):
            if any(p.sync_thread is not None and p.sync_thread.is_alive() for p in pods):
                return  # the s3-sync sidecar keeps the pod alive until its final sync
            st["completionTime"] = _now()
            st["replicaStatuses"]["Master"] = {"succeeded": 1, "selector": st["replicaStatuses"]["Master"]["selector"]}
            self._set_condition(job, "Succeeded", "PyTorchJobSucceeded", f"PyTorchJob {name} is successfully completed.")
            self._release(ns, name)

    def _set_condition(self, job, ctype, reason, message):
        conds = job["status"]["conditions"]
        for c in conds:
            c["status"] = "False" if c["type"] != ctype else c["status"]
        conds.append({"type": ctype, "status": "True", "reason": reason, "message": message,
                      "lastUpdateTime": _now(), "lastTransitionTime": _now()})
        self.history.append((job["metadata"]["name"], ctype))

    def _event(self, ns, obj_name, etype, reason, message):
        self.events.append({"metadata": {"namespace": ns, "name": f"{obj_name}.{len(self.events)}"},
                            "involvedObject": {"name": obj_name}, "type": etype, "reason": reason,
                            "message": message, "lastTimestamp": _now()})

    # ---- pods ----
    def _create_pods(self, ns, name, job):
        pods = []
        for rtype, rs in job["spec"]["pytorchReplicaSpecs"].items():
            for i in range(int(rs.get("replicas", 1))):
                pname = f"{name}-{rtype.lower()}-{i}"
                labels = dict(rs["template"]["metadata"].get("labels", {}))
                labels.update({JOB_NAME_LABEL: name, REPLICA_TYPE_LABEL: rtype.lower(), "training.kubeflow.org/replica-index": str(i)})
                if rtype == "Master":
                    labels[JOB_ROLE_LABEL] = "master"
                p = _Pod(pname, name, rtype.lower(), i, copy.deepcopy(rs["template"]["spec"]), labels)
                self.pods[(ns, pname)] = p
                self._event(ns, pname, "Normal", "Scheduled", f"Successfully assigned {ns}/{pname}")
                pods.append(p)
        nmaster_port = 29500 + (hash(name) % 2000)
        for p in pods:
            p.env_extra = {"PET_NNODES": str(len(pods)), "PET_NODE_RANK": str(0 if p.rtype == "master" else p.index + 1),
                           "PET_MASTER_ADDR": "127.0.0.1", "PET_MASTER_PORT": str(nmaster_port),
                           "WORLD_SIZE": str(len(pods)), "RANK": str(0 if p.rtype == "master" else p.index + 1),
                           "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(nmaster_port)}
            self._start_pod(ns, job, p)
        return pods

    def _wants_process(self, job) -> bool:
        if self.run_processes is True:
            return True
        if self.run_processes == "cpu":
            req = total_requests(job)
            return not any(k.endswith("/gpu") and v > 0 for k, v in req.items())
        return False

    def _start_pod(self, ns, job, p: _Pod):
        p.exit_code = None
        p.finish_time = None
        p.start_time = _now()
        p.phase = "Running"
        if p.workdir is None:
            p.workdir = os.path.join(self.workdir, ns, p.name)
            for sub in ("dataset", "artifacts"):
                os.makedirs(os.path.join(p.workdir, sub), exist_ok=True)
            self._run_init_containers(p)
        name = job["metadata"]["name"]
        if name in self._fail_next:
            self._fail_next.discard(name)
            p.append_log("Traceback (most recent call last): injected failure")
            p.exit_code, p.phase, p.finish_time = 1, "Failed", _now()
            return
        main = next(c for c in p.spec["containers"] if c["name"] == "pytorch")
        if self._wants_process(job):
            self._exec_main(p, main)
        else:
            p.sim_left = self.sim_ticks
            p.append_log("[fakecluster] simulated training container (no GPU on this host)")
        sidecar = next((c for c in p.spec["containers"] if c["name"] == "s3-sync"), None)
        if sidecar is not None and self.store is not None and (p.sync_thread is None or not p.sync_thread.is_alive()):
            p.sync_thread = threading.Thread(target=self._sidecar, args=(p, main, sidecar), daemon=True)
            p.sync_thread.start()

    def _mount(self, p: _Pod, main: dict, name: str) -> str | None:
        for vm in main.get("volumeMounts", []):
            if vm["name"] == name:
                return vm["mountPath"]
        return None

    def _localize(self, p: _Pod, main: dict, text: str) -> str:
        for vol, sub in (("model-checkpoint-volume", "artifacts"), ("dataset-volume", "dataset")):
            mp = self._mount(p, main, vol)
            if mp:
                text = text.replace(mp, os.path.join(p.workdir, sub))
        return text

    def _run_init_containers(self, p: _Pod):
        for ic in p.spec.get("initContainers", []):
            args = " ".join(ic.get("args", []))
            m = re.search(r"aws s3 cp (\S+) (\S+)", args)
            if m and self.store is not None:
                from ..blob.store import split_s3_uri

                bucket, key = split_s3_uri(m.group(1))
                dst = os.path.join(p.workdir, "dataset", os.path.basename(key))
                try:
                    self.store.get_file(bucket, key, dst)
                    p.append_log(f"[dataset-downloader] download: {m.group(1)} to {dst}")
                except Exception as e:
                    p.append_log(f"[dataset-downloader] failed: {e}")

    def _exec_main(self, p: _Pod, main: dict):
        body = self._localize(p, main, main["command"][-1])
        body = re.sub(r"(?<![\w/.-])python3?(?= )", shlex.quote(self.python), body)
        body = re.sub(r"(?<![\w/.-])torchrun(?= )", f"{shlex.quote(self.python)} -m torch.distributed.run", body)
        env = dict(os.environ)
        for e in main.get("env", []):
            env[e["name"]] = str(e.get("value", ""))
        env.update(getattr(p, "env_extra", {}))
        env.update(self._fault_env.get(p.job, {}))
        env["PYTHONPATH"] = REPO_ROOT + os.pathsep + env.get("PYTHONPATH", "")
        env["PYTHONUNBUFFERED"] = "1"
        env.pop("NCCL_DEBUG", None)
        p.proc = subprocess.Popen(["/bin/bash", "-c", body], stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                                  cwd=p.workdir, env=env, start_new_session=True)

        def pump(proc=p.proc):
            for raw in iter(proc.stdout.readline, b""):
                p.append_log(raw.decode("utf-8", errors="replace"))
            proc.wait()

        threading.Thread(target=pump, daemon=True).start()

    def _advance_pod(self, ns, job, p: _Pod):
        if p.exit_code is not None:
            if p.phase == "Running":
                p.phase = "Succeeded" if p.exit_code == 0 else "Failed"
                p.finish_time = p.finish_time or _now()
            return
        if p.proc is not None:
            rc = p.proc.poll()
            if rc is not None:
                p.exit_code = rc if rc >= 0 else 128 - rc
                p.phase = "Succeeded" if p.exit_code == 0 else "Failed"
                p.finish_time = _now()
                p.proc = None
            return
        # simulated container
        if p.sim_left > 0:
            step = self.sim_ticks - p.sim_left
            p.append_log(f"Epoch 0 | step {step + 1}/{self.sim_ticks} | loss {2.0 / (step + 1):.4f} | simulated")
            if p.rtype == "master":
                self._write_sim_artifacts(p, job, step + 1)
            p.sim_left -= 1
        else:
            p.exit_code = 0
            p.phase = "Succeeded"
            p.finish_time = _now()
            p.append_log("Training complete")

    def _write_sim_artifacts(self, p: _Pod, job, steps):
        art = os.path.join(p.workdir, "artifacts")
        with open(os.path.join(art, "metrics.csv"), "w") as f:
            f.write("epoch,step,loss,tokens_per_sec\n")
            for s in range(1, steps + 1):
                f.write(f"0,{s},{2.0 / s:.4f},{1000.0 * s:.1f}\n")
        if p.sim_left == 1:
            with open(os.path.join(art, "adapter_config.json"), "w") as f:
                f.write('{"peft_type": "LORA", "simulated": true}\n')

    def _kill(self, p: _Pod):
        if p.proc is not None and p.proc.poll() is None:
            try:
                os.killpg(p.proc.pid, signal.SIGKILL)
            except Exception:
                pass
        p.phase = "Failed" if p.exit_code is None else p.phase

    # ---- s3-sync sidecar ----
    def _sidecar(self, p: _Pod, main: dict, sidecar: dict):
        from ..blob.store import split_s3_uri

        script = " ".join(sidecar.get("args", []))
        m = re.search(r"aws s3 sync (\S+) (\S+)", script)
        if not m:
            return
        dest = m.group(2)
        pats = re.findall(r"--include '([^']+)'", script)
        # `aws s3 sync` filters: later ones win, so excludes written after the includes drop matches again
        first = script[script.index("--include"):].split(";", 1)[0] if pats else ""  # one `aws s3 sync` only
        tail_excl = re.findall(r"--exclude '([^']+)'", first)
        bucket, prefix = split_s3_uri(dest)
        art = os.path.join(p.workdir, "artifacts")
        done = os.path.join(art, "done.txt")
        failed = os.path.join(art, "failed.txt")
        synced: dict[str, float] = {}

        def sync_once():
            for fn in os.listdir(art):
                full = os.path.join(art, fn)
                if not os.path.isfile(full) or fn in ("done.txt", "failed.txt"):
                    continue
                if not any(fnmatch.fnmatch(fn, pat) for pat in pats):
                    continue
                if any(fnmatch.fnmatch(fn, pat) for pat in tail_excl):
                    continue
                mt = os.path.getmtime(full)
                if synced.get(fn) == mt:
                    continue
                try:
                    self.store.put_file(bucket, f"{prefix.rstrip('/')}/{fn}", full)
                    synced[fn] = mt
                except Exception as e:
                    p.append_log(f"[s3-sync] upload failed: {e}")

        fcount = 0
        while not self._stop.is_set():
            sync_once()
            if os.path.exists(done) or (p.proc is None and p.sim_left == 0 and p.exit_code == 0):
                break
            if os.path.exists(failed) or (p.exit_code not in (None, 0)):
                fcount += 1
                if fcount >= 3:
                    break
            else:
                fcount = 0
            time.sleep(self.sync_interval)
        sync_once()
