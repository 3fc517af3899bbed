"""Persistent document schemas (C11, Mongo side).

Collection documents are field-for-field compatible with the reference
(``/root/reference/app/schemas/db_schemas.py:10-136``) so an existing database keeps working -- including
the ``atrifacts_uri`` spelling (kept on purpose).
"""
from __future__ import annotations

from datetime import datetime
from enum import Enum
from typing import Any

from pydantic import BaseModel, BeforeValidator, ConfigDict, Field
from typing_extensions import Annotated


def _oid_to_str(v):
    return None if v is None else str(v)


PyObjectId = Annotated[str, BeforeValidator(_oid_to_str)]


class DatasetTypes(BaseModel):
    s3_uri: str = ""
    http_url: str = ""


class DatasetModel(BaseModel):
    model_config = ConfigDict(extra="allow", protected_namespaces=(), populate_by_name=True, from_attributes=True)
    id: PyObjectId | None = Field(default=None, alias="_id")
    user_id: str
    dataset: DatasetTypes
    dataset_name: str
    description: str = ""
    job_ref: list[str] = []
    created_at: datetime | None = None


class DatabaseStatusEnum(str, Enum):
    # running states
    queued = "queued"
    starting = "starting"
    restarting = "restarting"
    running = "running"
    # stopped states
    completed = "completed"
    failed = "failed"
    canceled = "canceled"
    error = "error"


class PromotionStatus(str, Enum):
    NOT_PROMOTED = "not_promoted"
    IN_PROGRESS = "in_progress"
    DELETING = "deleting"
    COMPLETED = "completed"
    FAILED = "failed"


class JobStatusMetadata(BaseModel):
    model_config = ConfigDict(extra="allow")
    start_time: datetime | None = None
    completion_time: datetime | None = None
    cancellation_time: datetime | None = None
    queue_pos: int | None = None


class JobStatus(BaseModel):
    model_config = ConfigDict(extra="allow", protected_namespaces=())
    user_id: str
    job_id: str
    job_name: str
    status: DatabaseStatusEnum
    promoted: PromotionStatus = PromotionStatus.NOT_PROMOTED
    created_at: datetime
    updated_at: datetime
    model_name: str
    device: str
    task: str
    framework: str
    arguments: dict[str, Any] | None = None
    dataset_id: str | None = None
    atrifacts_uri: str | None = None
    destination_uri: str | None = None
    dataset_name: str | None = None
    metadata: JobStatusMetadata | None = None


class JobsPage(BaseModel):
    items: list[JobStatus]
    total: int
    total_pages: int


class DatasetPage(BaseModel):
    items: list[DatasetModel]
    total: int
    total_pages: int


class MetricsDocument(BaseModel):
    model_config = ConfigDict(extra="ignore")
    user_id: str
    job_id: str
    job_name: str
    metrics: Any
