"""Worker / device configuration (C7).

``config.json`` (JSON with ``//`` comments) lists the worker types a job can be sent to: each has a
name, an optional Kueue LocalQueue (falling back to ``default_queue``), default resource
requests/limits, accelerator resource keys (whose COUNT is overridden by the model's
``accelerator_count``) and tolerations -- same schema as
``/root/reference/app/core/device_config.py:16-109`` and ``/root/reference/example.config.json``.

MI355X note: the accelerator resource key is ``amd.com/gpu`` (the AMD GPU device plugin), e.g.::

    {"name": "mi355x", "local_queue": "finetune-queue",
     "defaults": {"resources": {"requests": {"cpu": 16, "memory": "256Gi"}},
                  "accelerators": {"amd.com/gpu": 1}}}
"""
from __future__ import annotations

import json
import logging
from enum import Enum

from pydantic import BaseModel

logger = logging.getLogger("ftc.config")

AMD_GPU = "amd.com/gpu"


class ResourceDefaults(BaseModel):
    requests: dict[str, str | int] = {"cpu": 2, "memory": "1Gi"}
    limits: dict[str, str | int] = {}


class Toleration(BaseModel):
    """k8s toleration; the reference's {key, value, effect} (``device_config.py:21-24``) plus the
    optional ``operator`` (``Exists`` tolerations -- e.g. the AMD GPU operator's taint -- have no value)."""

    key: str
    value: str | None = None
    effect: str
    operator: str | None = None


class Defaults(BaseModel):
    resources: ResourceDefaults = ResourceDefaults()
    accelerators: dict[str, int] = {}

    def get_resources(self) -> dict[str, dict[str, str | int]]:
        return self.resources.model_dump()

    def get_accelerators(self) -> dict[str, int]:
        return self.accelerators


class Worker(BaseModel):
    name: str
    local_queue: str | None = None
    defaults: Defaults = Defaults()
    tolerations: list[Toleration] | None = None

    def get_tolerations(self) -> list[dict]:
        return [t.model_dump(exclude_none=True) for t in self.tolerations] if self.tolerations else []


class WorkersConfig(BaseModel):
    workers: list[Worker] = []
    default_queue: str | None = None

    def list_workers(self) -> list[str]:
        return [w.name for w in self.workers]

    def get_worker(self, name: str) -> Worker | None:
        for w in self.workers:
            if w.name == name:
                if self.default_queue and not w.local_queue:
                    return w.model_copy(update={"local_queue": self.default_queue})
                return w
        return None


class APIConfiguration(BaseModel):
    workers: WorkersConfig = WorkersConfig()

    def get_worker(self, name: str) -> Worker | None:
        return self.workers.get_worker(name)

    def list_workers(self) -> list[str]:
        return self.workers.list_workers()

    def device_enum(self):
        """Dynamic Enum of worker names, used for the API form (``DeviceTypes``)."""
        names = self.list_workers() or ["cpu"]
        return Enum("DeviceTypes", {n: n for n in names}, type=str)


def remove_json_comments(s: str) -> str:
    """Strip ``//`` comments outside strings.  Escapes are tracked, so a string ending in an escaped
    backslash (``"C:\\\\"``) closes where JSON says it does."""
    out, i, n, in_str, esc = [], 0, len(s), False, False
    while i < n:
        ch = s[i]
        if in_str:
            out.append(ch)
            if esc:
                esc = False
            elif ch == "\\":
                esc = True
            elif ch == '"':
                in_str = False
            i += 1
            continue
        if ch == '"':
            in_str = True
        elif s.startswith("//", i):
            j = s.find("\n", i)
            i = n if j < 0 else j
            continue
        out.append(ch)
        i += 1
    return "".join(out)


def parse_config(text: str) -> APIConfiguration:
    return APIConfiguration(workers=WorkersConfig(**json.loads(remove_json_comments(text))))


def load_config(path: str) -> APIConfiguration:
    try:
        with open(path) as f:
            cfg = parse_config(f.read())
        logger.debug("using worker configuration %s", path)
        return cfg
    except Exception:
        logger.error("error loading worker configuration (%s); create it to populate devices", path, exc_info=True)
        return APIConfiguration()


DEFAULT_CONFIG_JSON = """{
  // default LocalQueue for workers that name none
  "default_queue": "finetune-queue",
  "workers": [
    {"name": "cpu", "local_queue": "finetune-queue",
     "defaults": {"resources": {"requests": {"cpu": 2, "memory": "2Gi"}}}},
    {"name": "mi355x", "local_queue": "finetune-queue",
     "defaults": {"resources": {"requests": {"cpu": 16, "memory": "256Gi"}},
                  "accelerators": {"amd.com/gpu": 1}},
     "tolerations": [{"key": "amd.com/gpu", "value": "present", "effect": "NoSchedule"}]}
  ]
}"""
