"""Fine-tune job specification (C8): the pydantic contract a model author implements.

Field names, defaults and validation match ``/root/reference/app/models/base/finetuning.py:8-145`` so
model files written for the reference load unchanged (the API form, the Mongo documents and the
PyTorchJob manifest all derive from these fields).  MI355X-specific defaults live in the concrete
model specs (``spec/models``), not here.

``__init_subclass__`` rejects subclasses that re-declare a base field with an incompatible type
(e.g. ``accelerator_count: str``) -- the same guard as the reference, implemented by comparing the
declared annotation with the base annotation structurally.
"""
from __future__ import annotations

import shlex

from abc import ABC, abstractmethod
from enum import Enum
from typing import Any, get_args, get_origin

from pydantic import BaseModel, ConfigDict, Field


class TrainingTask(Enum):
    REGRESSION = "regression"
    CLASSIFICATION = "classification"
    MULTITASK_CLASSIFICATION = "multitask_classification"
    # [new] language-model fine-tuning tasks for the MI355X worker runtime
    CAUSAL_LM = "causal_lm"


class TrainingFramework(Enum):
    PYTORCH = "pytorch"
    TENSORFLOW = "tensorflow"


class TrainingArguments(BaseModel):
    """Per-model training flags; JSON-schema ``properties`` become the UI form."""

    model_config = ConfigDict(extra="ignore")


class TrainingResources(BaseModel):
    model_config = ConfigDict(extra="forbid")
    requests: dict[str, str | int]
    limits: dict[str, str | int] = {}


class TrainingDataset(BaseModel):
    model_config = ConfigDict(extra="forbid")
    description: str = Field(default="")
    dataset_required: bool = Field(default=False, description="Whether a dataset is required for training")
    dataset_name: str = Field(default="", description="Name of dataset file from api. set at runtime.")


def _types_compatible(base: Any, child: Any) -> bool:
    if child is base:
        return True
    bo, co = get_origin(base), get_origin(child)
    if bo or co:
        return bo == co and set(get_args(base)) == set(get_args(child))
    if isinstance(base, type) and isinstance(child, type):
        return issubclass(child, base)
    return base == child


class BaseFineTuneModel(BaseModel, ABC):
    model_config = ConfigDict(extra="ignore", protected_namespaces=())

    # identity / image
    name: str = Field(..., min_length=4, pattern=r"^[a-zA-Z0-9._@-]+$")
    inference_name: str | None = Field(default=None, description="Name of the model to be used for inference")
    image: str
    image_pull_secret: str | None = None
    command: list[str]
    framework: TrainingFramework
    task: TrainingTask
    description: str = ""
    project_url: str = ""

    # mounts
    checkpoint_mount: str = Field(default="/data/artifacts",
                                  description="Mount point for storing results. Best not to change this.")
    dataset_mount: str = Field(default="/data/dataset",
                               description="Mount point for storing dataset. Best not to change this.")
    dataset_info: TrainingDataset = TrainingDataset()
    device_types: list[str] = Field(default=["cpu"],
                                    description="Node type to run on based on taint toleration. Default 'cpu'")
    resources: TrainingResources = TrainingResources(requests={"cpu": 2, "memory": "1Gi"})
    accelerator_count: int = Field(default=1, ge=1, description="Number of gpu devices to use for training per worker")
    cluster_nodes: int = Field(default=1, ge=1, description="Total number of workers for training")
    store_asset_patterns: list[str] = Field(default=["*.json", "*.yaml", "*.csv", "*.pt", "*.ckpt"],
                                            description="Pattern match a list of files to store.")
    promotion_path: str = Field(default="", description="s3 prefix to upload artifacts "
                                                        "(inference path `domain/algorithm_name/algorithm_application`)")

    training_arguments: TrainingArguments

    @abstractmethod
    def run_cmd(self) -> list[str]:
        """The container command (``command`` with the rendered training flags appended)."""

    @classmethod
    def __init_subclass__(cls, **kwargs):
        super().__init_subclass__(**kwargs)
        declared = cls.__dict__.get("__annotations__", {})
        for fname, finfo in BaseFineTuneModel.model_fields.items():
            if fname not in declared:
                continue
            child_t = declared[fname]
            if isinstance(child_t, str):  # postponed annotations: resolve what we can
                try:
                    child_t = eval(child_t, vars(__import__(cls.__module__, fromlist=["*"])), {})  # noqa: S307
                except Exception:
                    continue
            if not _types_compatible(finfo.annotation, child_t):
                raise TypeError(f"Field '{fname}' in {cls.__name__} must have type {finfo.annotation}, got {child_t}")

    # ---- helpers shared by the concrete specs ----
    def append_args(self, args: list[str]) -> list[str]:
        """``command`` with ``args`` appended to its last element, plus the mount flags (the
        controller <-> trainer contract: ``--dataset_path`` / ``--checkpoint_path``).  Each element of
        ``args`` is ONE argument and is shell-quoted: the last element runs under ``sh -c``, and
        argument values come from the user's form (a ``--target-column=x; curl ...`` stays one word)."""
        cmd = list(self.command)
        tail = list(args) + [f"--dataset_path={self.dataset_mount}", f"--checkpoint_path={self.checkpoint_mount}"]
        cmd[-1] = (cmd[-1] + " " + " ".join(shlex.quote(str(a)) for a in tail)).strip()
        return cmd
