"""Queue position and pod diagnostics (C18).

* ``kueue_pending(kube, ns)`` -- PyTorchJob names whose Kueue ``Workload`` has ``QuotaReserved=False``,
  oldest first (``/root/reference/app/utils/kueue_helpers.py:19-46``); workloads already ``Finished``
  are skipped (a failed job stays on the cluster and must not hold a queue slot ahead of new ones);
* ``kubeflow_suspended(kube, ns)`` -- fallback ordering from the jobs' own ``Suspended`` condition.
  The reference compares ``type.lower()`` with ``"Suspended"`` and therefore never matches
  (``kueue_helpers.py:92``); fixed here.
* ``pod_events`` / ``pod_status`` -- the admin poll payload (``/root/reference/app/utils/kube_helpers.py:26-95``).
"""
from __future__ import annotations

import datetime as _dt
import logging

from .client import KubeClient

logger = logging.getLogger("ftc.k8s")


def kueue_pending(kube: KubeClient, namespace: str) -> list[str]:
    pending = []
    for wl in kube.list_workloads(namespace):
        md = wl.get("metadata", {})
        owners = md.get("ownerReferences") or []
        job = owners[0].get("name") if owners else None
        created = md.get("creationTimestamp", "")
        if not job or not created:
            continue
        conds = (wl.get("status") or {}).get("conditions", [])
        if any(c.get("type") == "Finished" and c.get("status") == "True" for c in conds):
            continue  # a finished workload (e.g. of a failed job the monitor keeps) is not queued
        if any(c.get("type") == "QuotaReserved" and c.get("status") == "False" for c in conds):
            pending.append((created, md.get("_seq", 0), job))
    pending.sort()
    return [j for _, _, j in pending]


def kueue_position(kube: KubeClient, namespace: str, job_id: str) -> int | None:
    q = kueue_pending(kube, namespace)
    return q.index(job_id) + 1 if job_id in q else None


def kubeflow_suspended(kube: KubeClient, namespace: str) -> list[str]:
    jobs = []
    for j in kube.list_pytorchjobs(namespace):
        conds = (j.get("status") or {}).get("conditions") or []
        if conds and conds[-1].get("type", "").lower() == "suspended":
            jobs.append((j["metadata"].get("creationTimestamp", ""), j["metadata"]["name"]))
    jobs.sort()
    return [n for _, n in jobs]


def queue_positions(kube: KubeClient, namespace: str) -> dict[str, int]:
    try:
        order = kueue_pending(kube, namespace)
    except Exception:
        logger.exception("kueue queue fetch failed, falling back to Kubeflow ordering")
        try:
            order = kubeflow_suspended(kube, namespace)
        except Exception as e:
            logger.error("failed to get queue information: %s", e)
            return {}
    return {job: i + 1 for i, job in enumerate(order)}


def _first_pod(kube: KubeClient, namespace: str, selector: str) -> dict | None:
    pods = kube.list_pods(namespace, selector)
    return pods[0] if pods else None


def pod_events(kube: KubeClient, namespace: str, selector: str) -> list[dict]:
    pod = _first_pod(kube, namespace, selector)
    if not pod:
        return []
    name = pod["metadata"]["name"]
    return [e for e in kube.list_events(namespace) if (e.get("involvedObject") or {}).get("name") == name]


def _parse_ts(s):
    if not s:
        return None
    if isinstance(s, _dt.datetime):
        return s
    return _dt.datetime.fromisoformat(str(s).replace("Z", "+00:00"))


def pod_status(kube: KubeClient, namespace: str, selector: str) -> dict | None:
    try:
        pod = _first_pod(kube, namespace, selector)
        if not pod:
            return None
        st = kube.read_pod(namespace, pod["metadata"]["name"]).get("status", {})
        cstats = st.get("containerStatuses") or []
        if not cstats:
            return None
        start = _parse_ts(st.get("startTime"))
        info = {"restart_count": 0, "start_time": start.isoformat() if start else None}
        for cs in cstats:
            info["restart_count"] += int(cs.get("restartCount", 0))
            state = cs.get("state") or {}
            if state.get("terminated"):
                fin = _parse_ts(state["terminated"].get("finishedAt"))
                if fin:
                    info["completion_time"] = fin.isoformat()
                    if start:
                        info["elapsed_time"] = f"{(fin - start).total_seconds():.1f}s"
            elif state.get("waiting"):
                info.update({"message": state["waiting"].get("message"), "reason": state["waiting"].get("reason"),
                             "status": cs.get("ready")})
        return info
    except Exception as e:
        logger.error("pod status failed: %s", e)
        return None
