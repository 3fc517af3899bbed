"""Control-plane settings (C17).

Same variable names, defaults and ``.env`` precedence as the reference
(``/root/reference/app/core/config.py:16-90``, template ``.env.example``): values from ``./.env``,
overridden by process environment variables.  Differences, per SURVEY.md §7.5:

* no import-time side effects -- ``get_settings()`` builds the object lazily and tests inject their own;
* AWS credentials are read ONCE (from ``AWS_ACCESS_KEY_ID`` / ``AWS_SECRET_ACCESS_KEY`` /
  ``AWS_REGION`` env vars if present, else from the Kubernetes Secret ``AWS_SECRET_NAME`` through the
  injected Kubernetes client) instead of three Secret reads on every property access;
* ``OPENBRIDGE_CLIENT_SECRET`` unset no longer crashes at import (the token validator is lazy).
"""
from __future__ import annotations

import base64
import json
import os
from typing import Any, Literal

from pydantic import BaseModel, ConfigDict, Field, SecretStr, field_validator


def _read_env_file(path: str) -> dict[str, str]:
    out: dict[str, str] = {}
    if not path or not os.path.exists(path):
        return out
    with open(path, encoding="utf-8") as f:
        for raw in f:
            line = raw.strip()
            if not line or line.startswith("#") or "=" not in line:
                continue
            k, v = line.split("=", 1)
            k = k.strip()
            if k.startswith("export "):
                k = k[len("export "):].strip()
            v = v.strip()
            # strip inline comments for unquoted values
            if v and v[0] in "\"'":
                q = v[0]
                end = v.find(q, 1)
                v = v[1:end] if end > 0 else v[1:]
            else:
                if " #" in v:
                    v = v.split(" #", 1)[0].rstrip()
            out[k] = v
    return out


class Settings(BaseModel):
    model_config = ConfigDict(extra="ignore")

    # server
    ENVIRONMENT: Literal["local", "staging", "production"] = "local"
    API_V1_STR: str = "/api/v1"
    LOG_STREAM_SEARCH_STRING: str | None = "Epoch"
    # cluster ("": the kube client's namespace -- the kubeconfig context's, or the service account's)
    NAMESPACE: str = ""
    # CORS
    FRONTEND_URL_CORS: list[str] = Field(default_factory=list)
    # security
    OPENBRIDGE_JWK_URL: str | None = None
    OPENBRIDGE_INTROSPECTION_URL: str | None = None
    OPENBRIDGE_CLIENT_ID: str | None = None
    OPENBRIDGE_CLIENT_SECRET: SecretStr | None = None
    OPENBRIDGE_API_KEY: SecretStr | None = None
    JWT_SECRET_KEY: str = ""
    JWT_ALGORITHM: str = "HS256"
    DEV_DISABLE_INTROSPECTION: bool = False
    # admin routes (/api/v1/admin/jobs/*, /admin/job/poll): with auth on, a caller is an admin when its
    # token's scp carries ADMIN_SCOPE or its subject is listed in ADMIN_USERS (comma-separated)
    ADMIN_SCOPE: str = "finetune:admin"
    ADMIN_USERS: list[str] = Field(default_factory=list)
    # worker config
    CONFIGURATION_FILE: str = "config.json"
    # database
    MONGODB_URL: str = "mongodb://localhost:27017"
    MONGODB_USERNAME: SecretStr | None = None
    MONGODB_PASSWORD: SecretStr | None = None
    MONGODB_DATABASE: str = "default"
    # job monitor
    JOB_MONITOR_INTERVAL: int = 2
    DEV_LOCAL_JOB_MONITOR: bool = False
    AWS_JOB_SYNC_INTERVAL: int = 60
    # aws
    S3_DEFAULT_DEPLOY_BUCKET: str = ""
    S3_BUCKET_NAME: str
    AWS_SECRET_NAME: str
    # [new] backends: "mongo" | "memory", "s3" | "local:<dir>", "kube" | "fake"
    STORE_BACKEND: str = "mongo"
    OBJECT_STORE: str = "s3"
    KUBE_BACKEND: str = "kube"
    S3_ENDPOINT_URL: str | None = None
    # [new] worker image used by the built-in MI355X model specs
    WORKER_IMAGE: str = "ghcr.io/finetune-controller-amd/worker-rocm:latest"
    CUSTOM_MODELS_DIR: str | None = None
    # [new] dataset_url submissions are fetched BY THE API SERVER: by default a URL (or a redirect)
    # that resolves to a loopback / private / link-local address (cluster services, the cloud metadata
    # endpoint) is refused; set true when datasets really live on an internal host
    DATASET_URL_ALLOW_PRIVATE: bool = False
    # [new] cached credentials (filled by load_aws_credentials)
    aws_access_key: SecretStr | None = None
    aws_secret_key: SecretStr | None = None
    aws_region: str | None = None

    @field_validator("FRONTEND_URL_CORS", mode="before")
    @classmethod
    def _cors(cls, v: Any):
        if isinstance(v, str):
            v = v.strip()
            if not v:
                return []
            if v.startswith("["):
                return json.loads(v)
            return [x.strip() for x in v.split(",") if x.strip()]
        return v

    @field_validator("OPENBRIDGE_JWK_URL", "OPENBRIDGE_INTROSPECTION_URL", "OPENBRIDGE_CLIENT_ID",
                     "OPENBRIDGE_CLIENT_SECRET", "OPENBRIDGE_API_KEY", "MONGODB_USERNAME", "MONGODB_PASSWORD",
                     mode="before")
    @classmethod
    def _empty_none(cls, v):
        return None if v == "" else v

    @classmethod
    def from_env(cls, env_file: str | None = "./.env", **overrides) -> "Settings":
        data: dict[str, Any] = {}
        data.update(_read_env_file(env_file) if env_file else {})
        for k in cls.model_fields:
            if k in os.environ:
                data[k] = os.environ[k]
        data.update(overrides)
        return cls(**data)

    # ---- AWS credentials, read once ----
    def load_aws_credentials(self, kube=None) -> "Settings":
        if self.aws_access_key is not None:
            return self
        ak = os.environ.get("AWS_ACCESS_KEY_ID")
        sk = os.environ.get("AWS_SECRET_ACCESS_KEY")
        rg = os.environ.get("AWS_REGION") or os.environ.get("AWS_DEFAULT_REGION")
        if (not ak or not sk) and kube is not None and self.AWS_SECRET_NAME:
            try:
                data = kube.read_secret(self.AWS_SECRET_NAME, self.NAMESPACE) or {}
                dec = {k: base64.b64decode(v).decode("utf-8") for k, v in data.items()}
                ak = ak or dec.get("AWS_ACCESS_KEY_ID")
                sk = sk or dec.get("AWS_SECRET_ACCESS_KEY")
                rg = rg or dec.get("AWS_REGION")
            except Exception:  # secret missing: fall back to ambient credentials
                pass
        self.aws_access_key = SecretStr(ak) if ak else None
        self.aws_secret_key = SecretStr(sk) if sk else None
        self.aws_region = rg or "us-east-1"
        return self

    @property
    def AWS_REGION(self) -> str:  # noqa: N802 - reference name
        return self.aws_region or os.environ.get("AWS_REGION", "us-east-1")


_settings: Settings | None = None


def get_settings() -> Settings:
    global _settings
    if _settings is None:
        _settings = Settings.from_env()
    return _settings


def set_settings(s: Settings | None) -> None:
    global _settings
    _settings = s
