"""Dependency container for the control plane.

Everything the reference keeps as import-time module singletons (``db_manager``, ``s3_handler``,
``api_instance``/``core_v1_api``, ``kubeflow_api``, ``validator``, ``JOB_MANIFESTS``,
``device_configuration``) lives on one ``AppContext`` built explicitly -- from settings in
production (``AppContext.from_settings``) or from fakes in tests / the local e2e path
(``AppContext.local``).
"""
from __future__ import annotations

import os
import tempfile
from dataclasses import dataclass, field

from .blob.handler import S3Handler
from .blob.store import LocalObjectStore, ObjectStore, make_object_store
from .core.config import Settings
from .core.device_config import APIConfiguration, load_config, parse_config, DEFAULT_CONFIG_JSON
from .k8s.client import HttpKubeClient, KubeClient
from .spec.registry import ModelRegistry
from .store.jobstore import JobStore


@dataclass
class AppContext:
    settings: Settings
    store: JobStore
    objects: ObjectStore
    kube: KubeClient
    registry: ModelRegistry
    devices: APIConfiguration
    s3: S3Handler = field(init=False)

    def __post_init__(self):
        self.s3 = S3Handler(self.objects, self.settings.S3_BUCKET_NAME)

    @property
    def namespace(self) -> str:
        return self.settings.NAMESPACE

    @classmethod
    def from_settings(cls, settings: Settings) -> "AppContext":
        if settings.KUBE_BACKEND == "fake":
            from .k8s.fake import FakeCluster

            kube: KubeClient = FakeCluster()
        else:
            kube = HttpKubeClient()
        if not settings.NAMESPACE:  # the kubeconfig context's / in-cluster service account's namespace
            settings.NAMESPACE = getattr(kube, "namespace", None) or "default"
        settings.load_aws_credentials(kube)
        objects = make_object_store(settings.OBJECT_STORE, settings)
        if settings.KUBE_BACKEND == "fake":  # the fake cluster's pods sync artifacts into the object store
            kube.store = objects
        registry = ModelRegistry()
        registry.load_custom(settings.CUSTOM_MODELS_DIR)
        return cls(settings, JobStore.from_settings(settings), objects, kube, registry,
                   load_config(settings.CONFIGURATION_FILE))

    @classmethod
    def local(cls, workdir: str | None = None, run_processes="cpu", config_json: str | None = None,
              **settings_overrides) -> "AppContext":
        """Everything in-process: memory store, local object store, FakeCluster (+ Kueue)."""
        from .k8s.fake import FakeCluster

        workdir = workdir or tempfile.mkdtemp(prefix="ftc-local-")
        s = dict(NAMESPACE="finetune-runner", S3_BUCKET_NAME="ftc-bucket", AWS_SECRET_NAME="aws-creds",
                 S3_DEFAULT_DEPLOY_BUCKET="ftc-deploy", STORE_BACKEND="memory",
                 OBJECT_STORE=f"local:{os.path.join(workdir, 's3')}", KUBE_BACKEND="fake",
                 JWT_SECRET_KEY="dev-secret", JOB_MONITOR_INTERVAL=1, AWS_JOB_SYNC_INTERVAL=1)
        s.update(settings_overrides)
        settings = Settings(**s)
        settings.aws_region = "us-east-1"
        objects = LocalObjectStore(os.path.join(workdir, "s3"))
        kube = FakeCluster(object_store=objects, run_processes=run_processes, workdir=os.path.join(workdir, "cluster"))
        return cls(settings, JobStore.memory(settings.MONGODB_DATABASE), objects, kube, ModelRegistry(),
                   parse_config(config_json or DEFAULT_CONFIG_JSON))
