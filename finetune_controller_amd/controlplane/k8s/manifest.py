"""PyTorchJob manifest builder (C6) -- a pure function of (job, worker, settings).

Produces a ``kubeflow.org/v1 PyTorchJob`` equivalent to the one the reference submits
(``/root/reference/app/jobs/kubeflow/PyTorchJobDeployer.py:20-262``): same labels, Kueue queue label +
``runPolicy.suspend``, resource merge, tolerations, dataset init container, ``pytorch`` training
container, ``s3-sync`` sidecar, Master + (N-1) Worker replicas, ``backoffLimit: 2`` and
``cleanPodPolicy: None``.  Deliberate differences:

* GPU fallback resource key is ``amd.com/gpu`` (AMD device plugin), not ``nvidia.com/gpu``;
* the training command is wrapped so a sentinel is ALWAYS written: ``done.txt`` on success, ``failed.txt``
  (exit code) on failure; the sidecar stops after the final sync on ``done.txt``, or once
  ``failed.txt`` has persisted for 3 sync periods (a restarted container removes it first).  The
  reference's sidecar loops forever when training fails;
* ``imagePullPolicy`` is set on the containers (it is not a PodSpec field);
* label values are sanitised to the Kubernetes label-value grammar (user ids may contain '@');
* a job with a dataset sets ``FTC_DATASET_EXPECTED=1`` on the training container: if the dataset
  download left the mount empty, the worker fails instead of training on synthetic tokens.
"""
from __future__ import annotations

import copy
import re
import shlex

from ..core.device_config import AMD_GPU, Worker
from ..schemas.jobs import JobInput

GROUP, VERSION, PLURAL, KIND = "kubeflow.org", "v1", "pytorchjobs", "PyTorchJob"
QUEUE_LABEL = "kueue.x-k8s.io/queue-name"
AWS_CLI_IMAGE = "amazon/aws-cli:latest"


def label_value(v) -> str:
    s = re.sub(r"[^A-Za-z0-9._-]", "_", str(v))[:63]
    return s.strip("._-") or "x"


def wrap_command(cmd: list[str], ckpt: str) -> list[str]:
    out = list(cmd)
    body = out[-1]
    q = shlex.quote
    out[-1] = (f"rm -f {q(ckpt + '/failed.txt')}; {body}; rc=$?; "
               f"if [ $rc -eq 0 ]; then touch {q(ckpt + '/done.txt')}; else echo $rc > {q(ckpt + '/failed.txt')}; fi; "
               f"exit $rc")
    return out


def sync_command(ckpt: str, dest: str, patterns: list[str], interval: int) -> str:
    q = shlex.quote  # every path / URI / pattern is quoted: none of them may be shell syntax
    inc = " ".join(f"--include {q(p)}" for p in patterns)
    # the worker's resume checkpoints (checkpoint_step*.pt: fp32 master weights + AdamW moments, ~96 GB
    # for an 8B full fine-tune) are read back from the pod's own volume only -- shipping every one to S3
    # would re-upload tens of GB per save for nothing; their .tmp halves are never synced either
    s = (f"aws s3 sync {q(ckpt)} {q(dest)} --exclude '*' {inc} --exclude 'done.txt' --exclude 'failed.txt' "
         f"--exclude 'checkpoint_step*.pt' --exclude '*.tmp'")
    return (f"f=0; while [ ! -f {q(ckpt + '/done.txt')} ]; do {s}; sleep {int(interval)}; "
            f"if [ -f {q(ckpt + '/failed.txt')} ]; then f=$((f+1)); [ $f -ge 3 ] && break; else f=0; fi; done; "
            f"{s}; ls -la {q(ckpt)}; echo 'Training finished. Exiting sidecar.'")


def merged_resources(job: JobInput, worker: Worker) -> dict:
    model = job.model
    res = worker.defaults.get_resources()
    # the model's requests/limits REPLACE the worker defaults (reference semantics)
    for k, v in model.resources.model_dump().items():
        res[k] = copy.deepcopy(v)
    res.setdefault("requests", {})
    res.setdefault("limits", {})
    acc = worker.defaults.get_accelerators()
    if acc:
        for key in acc:
            for section in ("requests", "limits"):
                res[section][key] = model.accelerator_count
    elif model.accelerator_count:
        res["requests"][AMD_GPU] = model.accelerator_count
        res["limits"][AMD_GPU] = model.accelerator_count
    return res


def build_pytorchjob_manifest(job: JobInput, worker: Worker, settings, namespace: str) -> dict:
    model = job.model
    if not (model.checkpoint_mount and settings.AWS_SECRET_NAME and settings.S3_BUCKET_NAME):
        raise ValueError("object storage is not configured (AWS_SECRET_NAME / S3_BUCKET_NAME)")
    region = getattr(settings, "AWS_REGION", None) or "us-east-1"
    command = wrap_command(model.run_cmd(), model.checkpoint_mount)
    labels = {
        "job.owner": label_value(job.user_id),
        "job.db-collection": label_value(settings.MONGODB_DATABASE),
        "job.model-name": label_value(job.model_name),
        "job.instance-type": label_value(job.device),
        "job.accelerators": str(int(model.accelerator_count) * int(model.cluster_nodes)),
        "job.nodes": str(model.cluster_nodes),
    }
    if worker.local_queue:
        labels[QUEUE_LABEL] = worker.local_queue
    aws_env = [{"name": "AWS_DEFAULT_REGION", "value": region}]
    aws_from = [{"secretRef": {"name": settings.AWS_SECRET_NAME}}]
    init_containers = []
    if job.s3_uri:
        init_containers.append({
            "name": "dataset-downloader",
            "image": AWS_CLI_IMAGE,
            "imagePullPolicy": "IfNotPresent",
            "command": ["/bin/sh", "-c"],
            # s3_uri ends in a user-supplied file name: quoted (the container holds the AWS secret)
            "args": [f"aws s3 cp {shlex.quote(job.s3_uri)} {shlex.quote(model.dataset_mount + '/')} ; echo 'done'; "
                     f"find {shlex.quote(model.dataset_mount)} -type f | wc -l; ls -la {shlex.quote(model.dataset_mount)}"],
            "volumeMounts": [{"name": "aws-credentials", "mountPath": "/root/.aws"},
                             {"name": "dataset-volume", "mountPath": model.dataset_mount}],
            "envFrom": aws_from,
            "env": aws_env,
        })
    # the job HAS a dataset: the worker must not fall back to synthetic tokens if the download left the
    # mount empty (its fallback is for dataset-optional specs submitted without one)
    expect_data = [{"name": "FTC_DATASET_EXPECTED", "value": "1"}] if job.s3_uri else []
    main = {
        "name": "pytorch",
        "image": model.image,
        "imagePullPolicy": "Always",
        "command": command,
        "volumeMounts": [
            {"name": "model-checkpoint-volume", "mountPath": model.checkpoint_mount, "readOnly": False},
            {"name": "dataset-volume", "mountPath": model.dataset_mount},
            {"name": "dshm", "mountPath": "/dev/shm"},
        ],
        "resources": merged_resources(job, worker),
        "env": [
            {"name": "HYDRA_FULL_ERROR", "value": "1"},
            {"name": "NCCL_DEBUG", "value": "INFO"},  # RCCL honours the NCCL_* variables
            {"name": "LOGLEVEL", "value": "DEBUG"},
            {"name": "PL_VERBOSE_LOGGING", "value": "1"},
        ] + expect_data,
    }
    sidecar = {
        "name": "s3-sync",
        "image": AWS_CLI_IMAGE,
        "imagePullPolicy": "IfNotPresent",
        "command": ["/bin/sh"],
        "args": ["-c", sync_command(model.checkpoint_mount, job.s3_artifacts_uri, model.store_asset_patterns,
                                    settings.AWS_JOB_SYNC_INTERVAL)],
        "volumeMounts": [{"name": "model-checkpoint-volume", "mountPath": model.checkpoint_mount, "readOnly": True},
                         {"name": "aws-credentials", "mountPath": "/root/.aws"}],
        "envFrom": aws_from,
        "env": aws_env,
    }
    pull = [{"name": model.image_pull_secret}] if model.image_pull_secret else []

    def pod_spec(containers):
        return {
            "imagePullSecrets": pull,
            "volumes": [
                {"name": "dataset-volume", "emptyDir": {}},
                {"name": "model-checkpoint-volume", "emptyDir": {}},
                {"name": "aws-credentials", "secret": {"secretName": settings.AWS_SECRET_NAME}},
                {"name": "dshm", "emptyDir": {"medium": "Memory"}},
            ],
            "initContainers": copy.deepcopy(init_containers),
            "containers": copy.deepcopy(containers),
            "tolerations": worker.get_tolerations(),
        }

    replicas = {
        "Master": {"replicas": 1, "restartPolicy": "OnFailure",
                   "template": {"metadata": {"labels": dict(labels)}, "spec": pod_spec([main, sidecar])}},
    }
    if model.cluster_nodes > 1:
        replicas["Worker"] = {"replicas": model.cluster_nodes - 1, "restartPolicy": "OnFailure",
                              "template": {"metadata": {"labels": dict(labels)}, "spec": pod_spec([main])}}
    return {
        "apiVersion": f"{GROUP}/{VERSION}",
        "kind": KIND,
        "metadata": {"name": job.job_id, "namespace": namespace, "labels": labels},
        "spec": {
            "runPolicy": {"suspend": bool(worker.local_queue), "backoffLimit": 2, "cleanPodPolicy": "None"},
            "pytorchReplicaSpecs": replicas,
        },
    }


def total_requests(manifest: dict) -> dict[str, float]:
    """Aggregate resource requests of all replicas (used by the Kueue emulation for admission)."""
    from .quantity import parse_quantity

    tot: dict[str, float] = {}
    for rs in manifest["spec"]["pytorchReplicaSpecs"].values():
        n = int(rs.get("replicas", 1))
        for c in rs["template"]["spec"]["containers"]:
            for k, v in (c.get("resources", {}).get("requests") or {}).items():
                tot[k] = tot.get(k, 0.0) + n * parse_quantity(v)
    return tot
